"""AddressSanitizer + UndefinedBehaviorSanitizer over the host code that takes caller-supplied bytes:
the product's JSON decode (csrc/host/objects.cpp over json.hpp -- what ksg_pod_compile, ksg_add_node,
ksg_upsert_namespace, ksg_upsert_object and ksg_create parse) and the parity oracle (decode, cache events,
scheduling cycles), built with -fsanitize=address,undefined (tests/asan/Makefile) and driven by seeded
mutations of real objects: the reference's fixture pods / nodes and fuzz_gen's random clusters."""
import glob
import json
import os
import random
import subprocess

import pytest

from fuzz_gen import CONFIGS, PTS_DEFAULT_CONFIGS, namespaces, rand_cluster, rand_objects, rand_pod

HERE = os.path.dirname(os.path.abspath(__file__))
ASAN = os.path.join(HERE, "asan")
BIN = os.path.join(ASAN, "build", "fuzz_decode")


def _build():
    subprocess.check_call(["make", "-s", "-j8", "-C", ASAN])
    return BIN


def _corpus(path, seed):
    rng, _, nodes, existing, names = rand_cluster(seed, n_nodes=40, n_existing=30)
    docs = [("node", n) for n in nodes] + [("ns", n) for n in namespaces()]
    docs += [("pod", p) for p in existing[:10]] + [("pod", rand_pod(rng, k, names)) for k in range(40)]
    docs += [("obj", o) for o in rand_objects(rng, 6)] + [("config", c) for c in CONFIGS + PTS_DEFAULT_CONFIGS]
    for f in sorted(glob.glob(os.path.join(HERE, "golden", "*.json")))[:8]:  # the reference's fixtures
        for c in json.load(open(f))["cases"][:6]:
            docs += [("node", n) for n in c.get("nodes", [])[:3]]
            docs += [("pod", p) for p in ([c["pod"]] if isinstance(c.get("pod"), dict) else []) + c.get("existing", [])[:3]]
    with open(path, "w") as out:
        for kind, d in docs:
            out.write(kind + "\t" + json.dumps(d, separators=(",", ":")) + "\n")
    return len(docs)


@pytest.mark.parametrize("seed", [1, 2])
def test_decode_and_oracle_under_asan_ubsan(tmp_path, seed):
    exe = _build()
    corpus = tmp_path / "corpus.txt"
    n = _corpus(str(corpus), 6100 + seed)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, str(corpus), str(seed), "40"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:] + r.stderr[-6000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert f"{n * 41} documents" in r.stdout, r.stdout

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


EV_BIN = os.path.join(ASAN, "build", "cache_events")


def _events(path, seed, n_events=1500):
    """A seeded cache-event sequence: node adds (some of which re-add removed ones), updates that move nodes
    between zones or change their taints / images / labels, removals (ghost nodes while pods remain), bound pods,
    pod deletions, assumes of compiled pods on random nodes (some unknown: ghost NodeInfos) and their forgets,
    reserved-and-dropped pod-table slots, and mirror uploads with a snapshot-order check after them."""
    from fuzz_gen import rand_node
    rng, _, nodes, existing, names = rand_cluster(seed, n_nodes=120, n_existing=0)
    live, gone, pods, assumed = [], list(nodes), [], []
    out = []

    def js(o):
        return json.dumps(o, separators=(",", ":"))

    for k in range(n_events):
        r = rng.random()
        if (r < 0.18 or not live) and gone:
            n = gone.pop(rng.randrange(len(gone)))
            live.append(n)
            out.append(f"node\t{js(n)}")
        elif r < 0.28 and live:
            i = rng.randrange(len(live))
            n = rand_node(rng, int(live[i]["metadata"]["name"][1:]))  # same name, new zone / taints / labels
            live[i] = n
            out.append(f"upd\t{js(n)}")
        elif r < 0.34 and live:
            n = live.pop(rng.randrange(len(live)))
            gone.append(n)
            out.append(f"rmnode\t{n['metadata']['name']}")
        elif r < 0.52:
            p = rand_pod(rng, 200000 + k, names)
            p["spec"].get("affinity", {}).pop("nodeAffinity", None)
            p["spec"]["nodeName"] = rng.choice(names)
            pods.append(p["metadata"]["uid"])
            out.append(f"pod\t{js(p)}")
        elif r < 0.60 and pods:
            out.append(f"rmpod\t{pods.pop(rng.randrange(len(pods)))}")
        elif r < 0.76:
            p = rand_pod(rng, 300000 + k, names)
            uid = f"{p['metadata']['uid']}#a{k}"
            node = rng.choice(names) if rng.random() < 0.95 else f"ghost-{k}"
            assumed.append(uid)
            out.append(f"assume\t{js(p)}\t{node}\t{uid}")
        elif r < 0.84 and assumed:
            out.append(f"forget\t{assumed.pop(rng.randrange(len(assumed)))}")
        elif r < 0.88:
            out.append(f"drop\t{js(rand_pod(rng, 400000 + k, names))}")
        else:
            out.append("mirror")
    out.append("mirror")
    open(path, "w").write("\n".join(out) + "\n")
    return len(out)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_cache_shadow_and_pod_table_under_asan_ubsan(tmp_path, seed):
    """The product's cache shadow and pod table (cluster.cpp, podtable.cpp, with the mirror uploads' host staging)
    under ASan / UBSan with the HIP runtime stubbed over host memory (tests/asan/hip_host_stub.cpp), against the
    oracle: every event's outcome agrees and the snapshot order after every upload is the oracle's."""
    _build()
    ev = tmp_path / "events.txt"
    n = _events(str(ev), 7700 + seed)
    cfg = json.dumps(CONFIGS[seed % len(CONFIGS)])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([EV_BIN, str(ev), cfg], capture_output=True, text=True, env=env, timeout=600)
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.returncode == 0, (r.stdout[-2000:] + r.stderr[-4000:])
    assert f"{n} events" in r.stdout and "0 divergences" in r.stdout, r.stdout

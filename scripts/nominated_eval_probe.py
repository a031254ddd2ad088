"""Diagnostic: tests/test_gpu_nominated.py::test_random_nominations_match_oracle[100-eval] pod by pod, printing
where the evaluation output first differs from the oracle's (key, node indices, both values)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-kubernetes_amd"), os.path.join(ROOT, "tests")]
from fuzz_gen import namespaces, rand_cluster  # noqa: E402
from oracle_binding import oracle  # noqa: E402
from test_gpu_nominated import _stream  # noqa: E402
from ksg.native import Scheduler  # noqa: E402

pct, mode = 100, "eval"
rng, cfg, nodes, existing, names = rand_cluster(5150 + pct + len(mode), n_nodes=700, n_existing=150)
cfg = dict(cfg, percentageOfNodesToScore=pct)
g, o = Scheduler(cfg), oracle(cfg)
for b in (g, o):
    for ns in namespaces():
        b.upsert_namespace(ns)
    for nd in nodes:
        b.add_node(nd)
    for p in existing:
        b.add_pod(p)
pods = _stream(rng, names, 160)
bad = 0
for k, p in enumerate(pods):
    rg, eg = g.schedule_one(g.compile(p), assume=True, evaluate=True)
    ro, eo = o.schedule_one(o.compile(p), assume=True, evaluate=True)
    if eg != eo or rg.as_tuple() != ro.as_tuple():
        bad += 1
        print(f"pod {k}: nominated={p.get('status', {}).get('nominatedNodeName')} dev {rg.as_tuple()} oracle {ro.as_tuple()}")
        for key in eo:
            a, b = eg.get(key), eo[key]
            if a != b:
                if isinstance(b, list) and isinstance(a, list) and len(a) == len(b):
                    idx = [i for i in range(len(b)) if a[i] != b[i]]
                    print(f"   {key}: {len(idx)} differ, first {[(i, a[i], b[i]) for i in idx[:6]]}")
                else:
                    print(f"   {key}: dev {str(a)[:200]} oracle {str(b)[:200]}")
        if bad >= 4:
            break
print("done", bad)

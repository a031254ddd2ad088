"""Debug helper: replays test_sampling_sequences_match_oracle[k-seed] and dumps the first mismatch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-kubernetes_amd"), os.path.join(ROOT, "tests")]
from fuzz_gen import rand_cluster, rand_pod  # noqa: E402
from ksg.native import Scheduler  # noqa: E402
import test_gpu_parity as t  # noqa: E402

k, seed = int(sys.argv[1]), int(sys.argv[2])
pct, extra = t.SAMPLING[k]
rng, _, nodes, existing, names = rand_cluster(5000 + 10 * k + seed, n_nodes=[130, 257, 600][seed], n_existing=60)
g, o = t._pair(Scheduler, dict(extra, percentageOfNodesToScore=pct), nodes, existing)
for q in range(30):
    pod = rand_pod(rng, q, names)
    rg, eg = g.schedule_one(g.compile(pod), assume=True, evaluate=True)
    ro, eo = o.schedule_one(o.compile(pod), assume=True, evaluate=True)
    print(q, rg.as_tuple(), ro.as_tuple())
    if rg.as_tuple() != ro.as_tuple():
        fg = [i for i, c in enumerate(eg["node_code"]) if c == 0]
        fo = [i for i, c in enumerate(eo["node_code"]) if c == 0]
        print("gpu code-0 nodes", len(fg), fg[:40])
        print("oracle code-0 nodes", len(fo), fo[:40])
        import json
        print(json.dumps(pod))
        bad = [i for i, (a, b) in enumerate(zip(eg["node_code"], eo["node_code"])) if a != b]
        for i in bad[:3]:
            print("node", i, names[i] if i < len(names) else None, "gpu", eg["node_code"][i], eg["node_plugin"][i], hex(eg["node_reasons"][i]),
                  "oracle", eo["node_code"][i], eo["node_plugin"][i], hex(eo["node_reasons"][i]))
        print("node names order", g.node_names()[40:44])
        print("diff codes", [(i, a, b) for i, (a, b) in enumerate(zip(eg["node_code"], eo["node_code"])) if a != b][:20])
        break

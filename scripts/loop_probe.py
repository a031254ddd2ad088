"""Diagnostic: k_sched_loop per-phase stamps and pods/s for several workgroup counts (C2 shape)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402

nodes_n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
wgs = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0"])]
hetero = len(sys.argv) > 3 and sys.argv[3] == "hetero"
nodes, init, pods = synth.scheduling_basic(nodes_n, 1000, 3000, hetero=hetero)
for wg in wgs:
    s = Scheduler({"device": 0, "loopWorkgroups": wg, "loopStamps": True})
    for n in nodes:
        s.add_node(n)
    for p in init:
        s.add_pod(p)
    hs = [s.compile(p) for p in pods]
    s.schedule_batch(hs[:1000], assume=True)
    arr = s.batch_arrays(hs[1000:3000])
    t = time.perf_counter()
    s.schedule_batch_into(*arr, assume=True)
    dt = time.perf_counter() - t
    print(f"nodes {nodes_n} wg {wg}: {2000 / dt:.0f} pods/s, stats {s.kernel_stats()}", flush=True)
    s.close()

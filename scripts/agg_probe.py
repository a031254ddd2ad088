"""Diagnostic: k_agg_loop per-phase stamps (workgroup 0's view) and pods/s on the aggregation
workloads: python scripts/agg_probe.py c3|c4|c4-anti|c5|dts [loopWorkgroups]."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
wg = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dbg = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if wl == "c3":
    nodes, init, pods = synth.scheduling_c3(5000, 5000, 2000)
elif wl in ("c4", "c4-anti"):
    nodes, init, pods = synth.topology_spreading(15000, 15000, 2000, preferred_anti=wl == "c4-anti")
elif wl == "dts":
    nodes, init, pods, objects = synth.default_topology_spreading(5000, 5000, 2000)
else:
    nodes, init, pods = synth.mixed_cluster(100000, 10000, 2000)
s = Scheduler({"device": 0, "loopWorkgroups": wg, "loopStamps": True, "aggLoopDebug": dbg})
for ns in synth.namespaces() if hasattr(synth, "namespaces") else []:
    s.upsert_namespace(ns)
for ob in (objects if wl == "dts" else []):
    s.upsert_object(ob)
for n in nodes:
    s.add_node(n)
for p in init:
    s.add_pod(p)
hs = [s.compile(p) for p in pods]
s.schedule_batch(hs[:1000], assume=True)
t = time.perf_counter()
s.schedule_batch(hs[1000:2000], assume=True)
dt = time.perf_counter() - t
print(f"{wl} wg {wg}: {1000 / dt:.0f} pods/s, stats {s.kernel_stats()}", flush=True)
s.close()

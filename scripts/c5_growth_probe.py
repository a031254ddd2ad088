"""Diagnostic: C5 (mixed 100k-node cluster) batch by batch -- wall ms, the batch's kernel stats (avg ms per
pod, pods in a loop, kernel) and mirror re-layouts -- to show what changes as assumed pods accumulate.
python scripts/c5_growth_probe.py [batches] [nodes] [c5|c2|c3|dts|c4|c4-anti] [stamps]  (c2: SchedulingBasic, 1000 init
pods; c3 / dts / c4 / c4-anti: as many init pods as nodes;
stamps: loopStamps, the loops' per-phase breakdown of every batch on stderr)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 50
N = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
WL = sys.argv[3] if len(sys.argv) > 3 else "c5"
if WL == "c2":
    nodes, init, pods = synth.scheduling_basic(N, 1000, B * 1000)
elif WL == "c3":
    nodes, init, pods = synth.scheduling_c3(N, N, B * 1000)
elif WL == "dts":
    nodes, init, pods = synth.default_topology_spreading(N, N, B * 1000)
elif WL in ("c4", "c4-anti"):
    nodes, init, pods = synth.topology_spreading(N, N, B * 1000, preferred_anti=WL == "c4-anti")
else:
    nodes, init, pods = synth.mixed_cluster(N, N // 10, B * 1000)
s = Scheduler({"device": 0, "kernelTimingStride": 1, "loopStamps": "stamps" in sys.argv[4:]})
for n in nodes:
    s.add_node(n)
for p in init:
    s.add_pod(p)
hs = [s.compile(p) for p in pods]
arrs = [s.batch_arrays(hs[k:k + 1000]) for k in range(0, B * 1000, 1000)]
for b, a in enumerate(arrs):
    t = time.perf_counter()
    s.schedule_batch_into(*a, assume=True)
    dt = (time.perf_counter() - t) * 1e3
    ms, by, n, k = s.kernel_stats()
    print(f"batch {b:3d}: {dt:8.2f} ms  kernel {k} n={n} avg {ms * 1e3:.2f} us  relayouts {s.relayouts()}", flush=True)
s.close()

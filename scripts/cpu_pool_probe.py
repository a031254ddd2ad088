"""Diagnostic: the oracle CPU baseline's scaling on this host -- pods/s and per-section us per pod for
1 thread and for 16 threads under each pool setting (spin before parking, NormalizeScore/weights on
the pool or not), C2 (5000 nodes) and C1 (500 nodes) shapes; `c3` / `c4`: those shapes over thread counts
and spins."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from ksg import synth  # noqa: E402

if sys.argv[1:2] in (["c3"], ["c4"]):  # pod-table shapes: threads x spin
    if sys.argv[1] == "c3":
        nodes, init, pods = synth.scheduling_c3(5000, 5000, 3000)
    else:
        nodes, init, pods = synth.topology_spreading(15000, 15000, 3000)
    for th, spin in ((1, 0), (8, 50), (8, 1000), (12, 1000), (16, 50), (16, 1000), (16, 5000)):
        v, done, dt, _ = bench.cpu_baseline(nodes, init, pods, 2.0, threads=th, extra={"cpuSpinUs": spin})
        print(json.dumps({"workload": sys.argv[1], "threads": th, "spin_us": spin, "pods_s": round(v),
                          "sections": bench.cpu_baseline.breakdown}), flush=True)
    sys.exit(0)
for n_nodes, n_init in ((5000, 1000), (500, 500)):
    nodes, init, pods = synth.scheduling_basic(n_nodes, n_init, 3000)
    v, done, dt, _ = bench.cpu_baseline(nodes, init, pods, 3.0, threads=1)
    print(json.dumps({"nodes": n_nodes, "threads": 1, "pods_s": round(v), "sections": bench.cpu_baseline.breakdown}),
          flush=True)
    for spin in (0, 20, 50, 100, 300):
        for pw in (False, True):
            v, done, dt, _ = bench.cpu_baseline(nodes, init, pods, 2.0, threads=16,
                                                extra={"cpuSpinUs": spin, "cpuParallelWeights": pw})
            print(json.dumps({"nodes": n_nodes, "threads": 16, "spin_us": spin, "parallel_weights": pw,
                              "pods_s": round(v), "sections": bench.cpu_baseline.breakdown}), flush=True)

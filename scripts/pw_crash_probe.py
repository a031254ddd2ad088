import sys
import os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "kubernetes-kubernetes_amd")); sys.path.insert(0, os.path.join(R, "tests"))
import bench
from ksg import synth
nodes, init, pods = synth.scheduling_basic(5000, 1000, 600)
for rep in range(6):
    for spin in (0, 20):
        v, done, dt, _ = bench.cpu_baseline(nodes, init, pods, 0.5, threads=16, extra={"cpuSpinUs": spin, "cpuParallelWeights": True})
        print(rep, spin, round(v), flush=True)

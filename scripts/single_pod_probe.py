"""Latency of one ksg_schedule_one call (the per-pod API a kube-scheduler binding calls from its
scheduling goroutine) on SchedulingBasic at 5000 nodes: the resident loop (default), the launch path,
against a ksg_schedule_batch of the same pods.  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg.synth import scheduling_basic  # noqa: E402


def run(cfg, n_pods=2000, batch=False):
    nodes, init, pods = scheduling_basic(5000, 1000, n_pods + 200)
    s = Scheduler(cfg)
    for n in nodes:
        s.add_node(n)
    for p in init:
        s.add_pod(p)
    hs = [s.compile(p) for p in pods]
    for h in hs[:200]:  # warm-up
        s.schedule_one(h, assume=True)
    t0 = time.perf_counter()
    if batch:
        s.schedule_batch(hs[200:], assume=True)
    else:
        for h in hs[200:]:
            s.schedule_one(h, assume=True)
    dt = time.perf_counter() - t0
    s.close()
    return dt / n_pods * 1e6


if sys.argv[1:] == ["stamps"]:  # the resident call's host / device split (printed at the loop's stop)
    print(json.dumps({"single_resident_us": round(run({"loopStamps": True}), 1)}))
    sys.exit(0)
out = {"single_resident_us": round(run({}), 1),
       "single_resident_pct0_us": round(run({"percentageOfNodesToScore": 0}), 1),
       "single_launch_us": round(run({"residentLoop": False}), 1),
       "single_launch_no_loop_us": round(run({"residentLoop": False, "persistentLoop": False}), 1),
       "batch_us_per_pod": round(run({}, batch=True), 2)}
print(json.dumps(out))

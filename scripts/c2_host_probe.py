"""Diagnostic: where a C2 step's time goes outside k_sched_loop.  Per-step wall time with every loop
launch timed by events (loopTimingStride 1) and with none (0), then one batch with loopStamps for
the host breakdown (chunk-0 compile, slot reservation, settle)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402

B, STEPS = 1000, 5
nodes, init, pods = synth.scheduling_basic(5000, 1000, B * (STEPS + 1))


def run(cfg, label):
    s = Scheduler(dict({"device": 0}, **cfg))
    for n in nodes:
        s.add_node(n)
    for p in init:
        s.add_pod(p)
    hs = [s.compile(p) for p in pods]
    s.schedule_batch(hs[:B], assume=True)
    arrs = [s.batch_arrays(hs[B * (k + 1):B * (k + 2)]) for k in range(STEPS)]
    ts = []
    for a in arrs:
        t = time.perf_counter()
        s.schedule_batch_into(*a, assume=True)
        ts.append(time.perf_counter() - t)
    st = s.kernel_stats()
    print(f"{label}: us per pod per step {[round(1e6 * x / B, 3) for x in ts]}  "
          f"mean {1e6 * sum(ts) / (B * STEPS):.3f}  kernel us/pod {1000 * st[0]:.3f}", flush=True)
    s.close()


if sys.argv[1:] == ["chunk"]:
    for rep in range(2):
        for fc in (64, 32, 16):
            run({"pipelineFirstChunk": fc}, f"pipelineFirstChunk {fc}")
    sys.exit(0)
if sys.argv[1:] == ["wavemap"]:
    for rep in range(2):
        for wm in (0, 1, 2):
            run({"loopWaveMap": wm}, f"loopWaveMap {wm}")
    for wm in (0, 1, 2):
        run({"loopWaveMap": wm, "loopStamps": True}, f"loopWaveMap {wm} stamps")
    sys.exit(0)
if sys.argv[1:] != ["stamps"]:
    run({"loopTimingStride": 1}, "events on every loop launch")
    run({"loopTimingStride": 0}, "no loop events")
    run({"loopTimingStride": 1}, "events on every loop launch (again)")
    run({"loopTimingStride": 3}, "events on every 3rd loop launch")
run({"loopStamps": True}, "loopStamps")

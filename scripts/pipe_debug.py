"""Debug helper: first mismatches of the pipeline re-layout stream against the oracle."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-kubernetes_amd"), os.path.join(ROOT, "tests")]
import test_gpu_parity as t  # noqa: E402
from ksg.native import Scheduler  # noqa: E402
from ksg.objects import PodW  # noqa: E402

nodes = t._pipeline_cluster()
pods = []
for k in range(700):
    p = PodW(f"p{k}", uid=f"p{k}").req({"cpu": "100m", "memory": "200Mi"})
    if k >= 300 and k % 5 == 0:
        p = p.node_selector({f"k{(k // 10) % 12}": f"v{k % 4}"} if k % 2 else {"tier": f"t{k % 3}"})
    pods.append(p.obj())
g, o = t._pair(lambda c: Scheduler(dict(c, loopStamps=True)), {}, nodes, [])
rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
bad = 0
for k, p in enumerate(pods):
    ro, _ = o.schedule_one(o.compile(p), assume=True)
    if rs[k].as_tuple() != ro.as_tuple():
        print(k, "gpu", rs[k].as_tuple(), "oracle", ro.as_tuple())
        bad += 1
        if bad > 12:
            break

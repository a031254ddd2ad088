import os, sys, time
sys.path.insert(0, "kubernetes-kubernetes_amd")
from ksg.native import Scheduler
from ksg.synth import scheduling_basic
nodes, init, pods = scheduling_basic(5000, 1000, 300)
for cfg in ({"loopStamps": True}, {"loopStamps": True, "persistentLoop": False}):
    s = Scheduler(cfg)
    for n in nodes: s.add_node(n)
    for p in init: s.add_pod(p)
    hs = [s.compile(p) for p in pods]
    for h in hs[:100]: s.schedule_one(h, assume=True)
    sys.stderr.write("---- %s\n" % cfg)
    for h in hs[100:110]: s.schedule_one(h, assume=True)
    t0 = time.perf_counter()
    for h in hs[110:300]: s.schedule_one(h, assume=False)
    sys.stderr.write("no-assume us %.1f\n" % ((time.perf_counter()-t0)/190*1e6))

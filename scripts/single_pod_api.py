"""200 single-pod ksg_schedule_one calls (SchedulingBasic, 5000 nodes) for a HIP API trace."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler
from ksg.synth import scheduling_basic
nodes, init, pods = scheduling_basic(5000, 1000, 300)
s = Scheduler({})
for n in nodes:
    s.add_node(n)
for p in init:
    s.add_pod(p)
hs = [s.compile(p) for p in pods]
for h in hs:
    s.schedule_one(h, assume=True)

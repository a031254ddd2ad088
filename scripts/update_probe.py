"""Diagnostic: cost of Cache.UpdateNode on the device mirror -- in place (same position, same taint /
image counts) against the full re-layout -- on the C5-sized cluster (100k nodes)."""
import copy
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
nodes, init, pods = synth.scheduling_basic(n_nodes, 1000, 2000)
s = Scheduler({"device": 0})
for n in nodes:
    s.add_node(n)
for p in init:
    s.add_pod(p)
hs = [s.compile(p) for p in pods]
s.schedule_batch(hs[:1000], assume=True)
upd = []
for k in range(200):
    n = copy.deepcopy(nodes[(k * 37) % n_nodes])
    n["status"]["allocatable"]["cpu"] = str(4 + k % 3)
    upd.append(n)
t = time.perf_counter()
for n in upd:
    s.update_node(n)
t_in = (time.perf_counter() - t) / len(upd)
t = time.perf_counter()
s.schedule_batch(hs[1000:1001], assume=True)
t_first = time.perf_counter() - t
# a layout change: the node moves to another zone, then the next cycle re-lays the mirror out
n = copy.deepcopy(nodes[5])
n["metadata"].setdefault("labels", {})["topology.kubernetes.io/zone"] = "zone-moved"
t = time.perf_counter()
s.update_node(n)
s.schedule_batch(hs[1001:1002], assume=True)
t_re = time.perf_counter() - t
print(f"{n_nodes} nodes: in-place UpdateNode {t_in * 1e6:.1f} us each (200 updates), next cycle {t_first * 1e3:.2f} ms; "
      f"zone change + next cycle (full re-layout) {t_re * 1e3:.2f} ms", flush=True)
s.close()

# node add / remove between cycles: re-laid out by gather (unchanged nodes' columns moved on the
# device) -- against the full rebuild (a new label key forces it: a new label column)
s = Scheduler({"device": 0})
for n in nodes:
    s.add_node(n)
for p in init:
    s.add_pod(p)
hs = [s.compile(p) for p in pods]
s.schedule_batch(hs[:1000], assume=True)
t_add = []
for k in range(5):
    n = copy.deepcopy(nodes[k])
    n["metadata"]["name"] = f"added-{k}"
    n["metadata"].setdefault("labels", {})["kubernetes.io/hostname"] = f"added-{k}"
    t = time.perf_counter()
    s.add_node(n)
    s.schedule_batch(hs[1000 + k:1001 + k], assume=True)
    t_add.append(time.perf_counter() - t)
t_rm = []
for k in range(5):
    t = time.perf_counter()
    s.remove_node(nodes[100 + 7 * k]["metadata"]["name"])
    s.schedule_batch(hs[1010 + k:1011 + k], assume=True)
    t_rm.append(time.perf_counter() - t)
f, g = s.relayouts()
nd = s.compare_mirror(sync=False)
print(f"{n_nodes} nodes: AddNode + next cycle {1e3 * sorted(t_add)[2]:.2f} ms, RemoveNode + next cycle "
      f"{1e3 * sorted(t_rm)[2]:.2f} ms (median of 5; re-layouts: {g} by gather, {f} full; mirror vs cache {nd})",
      flush=True)
s.close()

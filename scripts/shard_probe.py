"""Diagnostic: the node-sharded scheduler as W in-process ranks on one GPU (localGroup); pods/s and the loop's
per-pod time for each exchange mode.  python scripts/shard_probe.py 1,2d,2r,3d [c2|c4|c5]: SchedulingBasic with
5000 nodes per rank (c2), TopologySpreading with 5000 nodes and pods per rank (c4), the mixed cluster with
10000 nodes per rank (c5) -- weak scaling, one GPU's queues shared by every rank."""
import os
import sys
import threading
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402

WL = sys.argv[2] if len(sys.argv) > 2 else "c2"
PER = {"c2": 5000, "c4": 5000, "c5": 10000}[WL]
for world, dx in [(int(w.rstrip("dr")), w.endswith("d")) for w in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["2d", "2r"])]:
    if WL == "c4":
        nodes, init, pods = synth.topology_spreading(PER * world, PER * world, 3000)
    elif WL == "c5":
        nodes, init, pods = synth.mixed_cluster(PER * world, 1000 * world, 3000)
    else:
        nodes, init, pods = synth.scheduling_basic(PER * world, 1000 * world, 3000)
    name = f"p-{uuid.uuid4().hex[:6]}"
    ranks = []
    for r in range(world):
        cfg = {"device": 0, "deviceExchange": dx}
        if world > 1:
            cfg["distributed"] = {"worldSize": world, "rank": r, "localGroup": name}
        s = Scheduler(cfg)
        for n in nodes:
            s.add_node(n)
        for p in init:
            s.add_pod(p)
        ranks.append(s)
    hs = [[s.compile(p) for p in pods] for s in ranks]
    arrs = [[s.batch_arrays(h[k:k + 1000]) for k in range(0, 3000, 1000)] for s, h in zip(ranks, hs)]
    dts = [0.0] * world

    def work(r):
        ranks[r].schedule_batch_into(*arrs[r][0], assume=True)  # warmup
        t = time.perf_counter()
        for a in arrs[r][1:]:
            ranks[r].schedule_batch_into(*a, assume=True)
        dts[r] = time.perf_counter() - t

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = max(dts)
    print(f"{WL} world {world} {'device' if dx else 'all-reduce'} exchange, {PER * world} nodes: {2000 / dt:.0f} pods/s, "
          f"rank 0 stats {ranks[0].kernel_stats()}", flush=True)
    for s in ranks:
        s.close()

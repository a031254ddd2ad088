"""Diagnostic: test_c5_pipelined_batches_sharded_agg_loop at W = 3, repeated `reps` times in one process
(fresh groups), printing each rank's error -- the k_agg_loop give-up record names its first failure."""
import os
import sys
import threading
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from ksg.native import Scheduler  # noqa: E402
from ksg.synth import mixed_cluster  # noqa: E402
from fuzz_gen import namespaces  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
nodes, init, pods = mixed_cluster(6000, 1200, 1200)
for rep in range(reps):
    name = f"w-{uuid.uuid4().hex[:6]}"
    ranks = []
    for r in range(W):
        s = Scheduler({"deviceExchange": True, "device": 0,
                       "distributed": {"worldSize": W, "rank": r, "localGroup": name}})
        for ns in namespaces():
            s.upsert_namespace(ns)
        for n in nodes:
            s.add_node(n)
        for p in init:
            s.add_pod(p)
        ranks.append(s)
    hs = [[s.compile(p) for p in pods] for s in ranks]
    errs = []

    def work(r):
        try:
            for k in range(0, len(pods), 600):
                ranks[r].schedule_batch(hs[r][k:k + 600], assume=True)
        except Exception as e:
            errs.append((r, str(e)))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=200)
    print(f"rep {rep}: {'ok' if not errs else errs}", flush=True)
    for s in ranks:
        s.close()

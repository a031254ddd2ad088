"""Diagnostic: in-process device-exchange groups (localGroup, deviceExchange) formed one after another in ONE
process, each reporting per rank its loop give-ups / re-runs, the dominant kernel and the last error text
(which, after a recovered give-up, carries give_up_detail's missing participants per rank).

    python scripts/group_probe.py STEP[,STEP...]
      o      create one more unsharded context ("other") and keep it
      x      close the "other" contexts
      <W>    a W-rank group: SchedulingBasic hetero (1877 + 256 W nodes, 300 init, 600 pods, chunks of 300),
             closed again afterwards
      <W>k   the same group, kept open (closed by the next 'c')
      <W>r   the same group on the all-reduce path (deviceExchange off)
      c      close kept groups
The round-5 give-up sequence is  o,6,x,6  (test_group_loops_start_together_after_contexts_closed)."""
import os
import sys
import threading
import time
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
from ksg.native import Scheduler  # noqa: E402
from ksg import synth  # noqa: E402


def group(world, tag, dx=True):
    nodes, init, pods = synth.scheduling_basic(1877 + 256 * world, 300, 600, hetero=True)
    name = f"g-{uuid.uuid4().hex[:6]}"
    ranks = []
    for r in range(world):
        s = Scheduler({"device": 0, "deviceExchange": dx, "featureGates": {"OpportunisticBatching": False},
                       "distributed": {"worldSize": world, "rank": r, "localGroup": name}})
        for n in nodes:
            s.add_node(n)
        for p in init:
            s.add_pod(p)
        ranks.append(s)
    hs = [[s.compile(p) for p in pods] for s in ranks]
    out = [[] for _ in ranks]
    errs = []
    dts = [0.0] * world

    def work(r):
        try:
            t = time.perf_counter()
            for k in range(0, len(pods), 300):
                out[r].extend(x.as_tuple() for x in ranks[r].schedule_batch(hs[r][k:k + 300], assume=True))
            dts[r] = time.perf_counter() - t
        except Exception as e:
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    agree = all(o == out[0] for o in out)
    print(f"[{tag}] W={world} max {max(dts):.2f}s agree={agree} errs={errs}", flush=True)
    for r, s in enumerate(ranks):
        err = s.last_error()  # first: the other calls clear it
        print(f"   rank {r}: loop_stats={s.loop_stats()} kernel={s.kernel_stats()[3]} shard={s.shard_range()} "
              f"err={err[:1500]!r}", flush=True)
    return ranks


others, kept = [], []
for k, st in enumerate(sys.argv[1].split(",")):
    tag = f"{k}:{st}"
    if st == "o":
        others.append(Scheduler({"device": 0}))
        print(f"[{tag}] other contexts: {len(others)}", flush=True)
    elif st == "x":
        for s in others:
            s.close()
        others = []
        print(f"[{tag}] closed other contexts", flush=True)
    elif st == "c":
        for g in kept:
            for s in g:
                s.close()
        kept = []
        print(f"[{tag}] closed kept groups", flush=True)
    else:
        keep = st.endswith("k")
        ranks = group(int(st.rstrip("kr")), tag, dx=not st.endswith("r"))
        if keep:
            kept.append(ranks)
        else:
            for s in ranks:
                s.close()

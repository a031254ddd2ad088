"""Repeat test_c5_mixed_sharded_agg_loop's workload (configs[4]'s mixed stream on 20 000 nodes, W in-process
ranks, device exchange) in fresh groups and report every rank's mismatches against the oracle, pod by pod --
which fields differ, on which ranks -- to characterise an intermittent mismatch (round 6: one suite run of six
saw rank 0 pod 2 with 76 fewer feasible nodes than the oracle, same node and score).

  python scripts/sharded_repeat_probe.py [world] [repeats]
"""
import os
import sys
import threading
import uuid

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from fuzz_gen import namespaces  # noqa: E402
from ksg.native import Scheduler  # noqa: E402
from ksg.synth import mixed_cluster  # noqa: E402
from oracle_binding import oracle  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    nodes, init, pods = mixed_cluster(20000, 2000, 240)
    cfg = {"deviceExchange": True, "featureGates": {"OpportunisticBatching": False}}
    o = oracle(cfg)
    for ns in namespaces():
        o.upsert_namespace(ns)
    for n in nodes:
        o.add_node(n)
    for p in init:
        o.add_pod(p)
    want = [o.schedule_one(o.compile(p), assume=True)[0].as_tuple() for p in pods]
    for rep in range(reps):
        name = f"p-{uuid.uuid4().hex[:8]}"
        ranks = []
        for r in range(world):
            s = Scheduler(dict(cfg, device=0, distributed={"worldSize": world, "rank": r, "localGroup": name}))
            for ns in namespaces():
                s.upsert_namespace(ns)
            for n in nodes:
                s.add_node(n)
            for p in init:
                s.add_pod(p)
            ranks.append(s)
        hs = [[s.compile(p) for p in pods] for s in ranks]
        out = [[] for _ in ranks]

        def work(r):
            for k in range(0, len(pods), 120):
                out[r].extend(x.as_tuple() for x in ranks[r].schedule_batch(hs[r][k:k + 120], assume=True))

        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        bad = []
        for k in range(len(pods)):
            for r in range(world):
                if out[r][k] != want[k]:
                    bad.append((k, r, out[r][k], want[k]))
        stats = [s.loop_stats() for s in ranks]
        kinds = {k: pods[k]["metadata"]["name"] for k, _, _, _ in bad}
        print(f"rep {rep}: {len(bad)} mismatches, loop stats {stats}", flush=True)
        for k, r, g, w in bad[:12]:
            print(f"   pod {k} ({kinds[k]}) rank {r}: got {g} want {w}", flush=True)
        for s in ranks:
            s.close()


if __name__ == "__main__":
    main()

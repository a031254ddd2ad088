import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "kubernetes-kubernetes_amd")
from fuzz_gen import namespaces, rand_cluster, rand_pod
from oracle_binding import oracle
from ksg.native import Scheduler
pass
for dbg in (0, 32):
    rng, cfg, nodes, existing, names = rand_cluster(1000, n_nodes=513, n_existing=100)
    bs = []
    for make, c in ((Scheduler, dict(cfg, aggLoopDebug=dbg, loopStamps=True)), (oracle, cfg)):
        b = make(c)
        for ns in namespaces(): b.upsert_namespace(ns)
        for n in nodes: b.add_node(n)
        for p in existing: b.add_pod(p)
        bs.append(b)
    g, o = bs
    pods = [rand_pod(rng, k, names) for k in range(50)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    bad = []
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        if rs[k].as_tuple() != ro.as_tuple(): bad.append((k, rs[k].as_tuple(), ro.as_tuple()))
        if False: print(k, rs[k].as_tuple(), ro.as_tuple(), "aff" if ("affinity" in p["spec"]) else "", "spread" if p["spec"].get("topologySpreadConstraints") else "", flush=True)
    print("debug", dbg, "mismatches", len(bad), bad[:3], flush=True)

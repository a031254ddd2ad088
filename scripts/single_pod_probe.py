"""Latency of one ksg_schedule_one call (the per-pod API a kube-scheduler binding calls from its
scheduling goroutine, schedule_one.go:67-192): the resident loops (default: k_sched_loop for node-local
pods, k_agg_loop for PodTopologySpread / InterPodAffinity pods), the launch path, and a
ksg_schedule_batch of the same pods.  Prints one JSON line per workload.

  python scripts/single_pod_probe.py [workload ...]     c2 (SchedulingBasic 5000 nodes, default), c2pct0,
                                                        dts (DefaultTopologySpreading), c4 (TopologySpreading
                                                        15000 nodes), c3, c3aff (C3's pod-affinity pods alone), c4-anti, c5 (100 000 nodes), c2big (SchedulingBasic at 100 000 nodes)
  python scripts/single_pod_probe.py stamps [workload]  the resident call's host / device split
  python scripts/single_pod_probe.py ab [workload]      resident variants (residentAhead, the doorbell relay, and
                                                        k_agg_loop's same-template shortcuts off: aggLoopDebug 8 / 12)
single_resident_us times the calls from Python (ctypes), single_resident_native_us from native code
(ksg_debug_schedule_calls), as a binding's goroutine issues them.
Every resident call's result is checked against the oracle (after timing), so a fast wrong answer
does not count.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from ksg import synth  # noqa: E402
from ksg.native import Scheduler  # noqa: E402


def cluster(wl, n_pods):
    objects = []
    if wl in ("c2", "c2pct0"):
        nodes, init, pods = synth.scheduling_basic(5000, 1000, n_pods)
    elif wl == "c2big":  # SchedulingBasic pods on 100 000 nodes
        nodes, init, pods = synth.scheduling_basic(100000, 1000, n_pods)
    elif wl == "dts":
        nodes, init, pods, objects = synth.default_topology_spreading(5000, 5000, n_pods)
    elif wl == "c3":
        nodes, init, pods = synth.scheduling_c3(5000, 5000, n_pods)
    elif wl == "c3aff":  # C3's cluster, the measured stream one template: pod-with-pod-affinity (own terms)
        nodes, init, _ = synth.scheduling_c3(5000, 5000, 0)
        pods = [synth.pod_with_pod_affinity(f"pod-{k}", "sched-1") for k in range(n_pods)]
    elif wl == "c5":
        nodes, init, pods = synth.mixed_cluster(100000, 10000, n_pods)
    else:
        nodes, init, pods = synth.topology_spreading(15000, 15000, n_pods, preferred_anti=wl == "c4-anti")
    return nodes, init, pods, objects


def run(wl, cfg, n_pods=2000, batch=False, check=False, native=False):
    nodes, init, pods, objects = cluster(wl, n_pods + 200)
    if wl == "c2pct0":
        cfg = dict(cfg, percentageOfNodesToScore=0)
    s = Scheduler(cfg)
    for ob in objects:
        s.upsert_object(ob)
    for n in nodes:
        s.add_node(n)
    for p in init:
        s.add_pod(p)
    hs = [s.compile(p) for p in pods]
    got = [s.schedule_one(h, assume=True)[0].as_tuple() for h in hs[:200]]  # warm-up
    t0 = time.perf_counter()
    if batch:
        got += [r.as_tuple() for r in s.schedule_batch(hs[200:], assume=True)]
    elif native:  # the calls from native code: no interpreter overhead per call
        rs, us = s.schedule_calls(hs[200:], assume=True)
        got += [r.as_tuple() for r in rs]
    else:
        for h in hs[200:]:
            got.append(s.schedule_one(h, assume=True)[0].as_tuple())
    dt = us * n_pods * 1e-6 if native else time.perf_counter() - t0
    kern = s.kernel_stats()[3]
    s.close()
    mism = None
    if check:
        from oracle_binding import oracle
        o = oracle(dict(percentageOfNodesToScore=0) if wl == "c2pct0" else {"cpuThreads": 16} if wl in ("c5", "c2big") else {})
        for ob in objects:
            o.upsert_object(ob)
        for n in nodes:
            o.add_node(n)
        for p in init:
            o.add_pod(p)
        mism = 0
        for k, p in enumerate(pods):
            if o.schedule_one(o.compile(p), assume=True)[0].as_tuple() != got[k]:
                mism += 1
    return dt / n_pods * 1e6, kern, mism


def main():
    args = sys.argv[1:]
    if args[:1] == ["ab"]:  # resident-loop variants, native calls, oracle-checked, interleaved twice on one box
        wl = args[1] if len(args) > 1 else "c2"
        variants = [("ahead+relay", {"ringRelayMinWorkgroups": 1}), ("ahead", {}),
                    ("relay", {"residentAhead": False, "ringRelayMinWorkgroups": 1}), ("neither", {"residentAhead": False}),
                    # k_agg_loop: every pod staged over PCIe (no RING_SAME / RING_TERMS), and no fold either
                    ("staged", {"aggLoopDebug": 8}), ("staged+gathered", {"aggLoopDebug": 12})]
        for rep in range(2):
            for name, cfg in variants:
                nus, _, nmism = run(wl, cfg, check=rep == 0, native=True)
                print(json.dumps({"workload": wl, "variant": name, "rep": rep, "single_resident_native_us": round(nus, 2),
                                  "native_oracle_mismatches": nmism}), flush=True)
        return
    if args[:1] == ["stamps"]:  # printed at the loop's stop
        wl = args[1] if len(args) > 1 else "c2"
        print(json.dumps({"workload": wl, "single_resident_us": round(run(wl, {"loopStamps": True})[0], 1),
                          "single_resident_native_us": round(run(wl, {"loopStamps": True}, native=True)[0], 1)}))
        return
    for wl in args or ["c2"]:
        us, kern, mism = run(wl, {}, check=True)
        nus, _, nmism = run(wl, {}, check=True, native=True)
        out = {"workload": wl, "single_resident_us": round(us, 1), "single_resident_native_us": round(nus, 1),
               "resident_kernel": kern, "oracle_mismatches": mism, "native_oracle_mismatches": nmism,
               "single_launch_us": round(run(wl, {"residentLoop": False})[0], 1),
               "batch_us_per_pod": round(run(wl, {}, batch=True)[0], 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

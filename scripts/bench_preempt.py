"""PreemptionBasic (scheduler_perf misc/performance-config.yaml:124-170) through ksg_preempt.

Cluster: N nodes of node-default.yaml (4 CPU, 32Gi, 110 pods), 4 low-priority pods per node
(pod-low-priority.yaml: 900m / 500Mi, priority 0), then M high-priority pods (pod-high-priority.yaml:
3000m / 500Mi, priority 10).  Per measured pod, the flow a scheduler runs:

  schedulingCycle -> FitError -> PostFilter (ksg_preempt: eligibility, the cycle's statuses, SelectVictimsOnNode
  on every potential node, candidate cut, pickOneNodeForPreemption) -> the victims' deletions arrive
  (ksg_remove_pod) -> the retried cycle binds the pod (ksg_schedule_one + assume)

Timed: the whole flow per pod, and ksg_preempt alone.  The oracle runs the same flow on the same
cluster for the first pods (a bounded CPU sample, one thread) and every preemption's result (node,
victims) is compared with it.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-kubernetes_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def node(i):
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": f"scheduler-perf-{i:05d}"}, "spec": {},
            "status": {"capacity": {"pods": "110", "cpu": "4", "memory": "32Gi"},
                       "allocatable": {"pods": "110", "cpu": "4", "memory": "32Gi"}}}


def pod(name, prio, cpu, node_name=None, start=None):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default", "uid": name},
         "spec": {"containers": [{"name": "pause", "image": "registry.k8s.io/pause:3.10.1",
                                  "ports": [{"containerPort": 80}],
                                  "resources": {"requests": {"cpu": cpu, "memory": "500Mi"},
                                                "limits": {"cpu": cpu, "memory": "500Mi"}}}]},
         "status": {}}
    if prio:
        p["spec"]["priority"] = prio
    if node_name:
        p["spec"]["nodeName"] = node_name
    if start is not None:
        p["status"]["startTime"] = f"2024-01-01T00:{start // 60 % 60:02d}:{start % 60:02d}Z"
    return p


def build(make, n_nodes):
    b = make({})
    for i in range(n_nodes):
        b.add_node(node(i))
    for i in range(n_nodes):
        for k in range(4):
            b.add_pod(pod(f"pod-{i}-{k}", 0, "900m", f"scheduler-perf-{i:05d}", start=(i * 4 + k) % 3600))
    return b


def flow(b, p, args):
    """One measured pod; returns (preempt seconds, nominated node, victims, bound node)."""
    h = b.compile(p)
    r, _ = b.schedule_one(h, assume=False)
    assert r.status == 2, f"{p['metadata']['name']}: expected a FitError, got status {r.status}"
    t0 = time.perf_counter()
    pr, d = b.preempt(h, args)
    t1 = time.perf_counter()
    for uid in d["victims"]:
        b.remove_pod(uid)
    r2, _ = b.schedule_one(h, assume=True)
    return t1 - t0, d.get("selected"), d["victims"], r2.node_index


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--pods", type=int, default=1000)
    ap.add_argument("--cpu-pods", type=int, default=100)
    a = ap.parse_args()
    from ksg.native import Scheduler
    from oracle_binding import oracle
    args = {"offset": 0, "now": 1704153600 * 10 ** 9}  # 2024-01-02: later than every startTime
    dev = build(Scheduler, a.nodes)
    pods = [pod(f"pod-high-priority-{q}", 10, "3000m") for q in range(a.pods)]
    # warm-up on a throwaway copy of the state would change it; the first pod is timed like the rest
    t0 = time.perf_counter()
    pre_s, dev_out = 0.0, []
    for q, p in enumerate(pods):
        args["offset"] = q * 7919
        dt, sel, vic, bound = flow(dev, p, args)
        pre_s += dt
        dev_out.append((sel, vic, bound))
    wall = time.perf_counter() - t0
    orc = build(oracle, a.nodes)
    t0 = time.perf_counter()
    ore_s, mism = 0.0, 0
    for q, p in enumerate(pods[:a.cpu_pods]):
        args["offset"] = q * 7919
        dt, sel, vic, bound = flow(orc, p, args)
        ore_s += dt
        mism += (sel, vic, bound) != dev_out[q]
    owall = time.perf_counter() - t0
    print(json.dumps({
        "metric": "PreemptionBasic preemptor pods/s (FitError cycle + PostFilter + victim deletions + bind)",
        "value": round(a.pods / wall, 1), "unit": "pods/s",
        "postfilter_us_per_pod": round(pre_s / a.pods * 1e6, 1),
        "config": {"workload": f"PreemptionBasic {a.nodes} nodes / {4 * a.nodes} low-priority pods / "
                               f"{a.pods} high-priority pods", "nodes": a.nodes},
        "cpu_baseline": {"value": round(a.cpu_pods / owall, 1), "unit": "pods/s", "cores": 1, "kind": "port",
                         "postfilter_us_per_pod": round(ore_s / a.cpu_pods * 1e6, 1),
                         "sample": f"the first {a.cpu_pods} measured pods, same flow, oracle/"},
        "parity": {"checked_pods": a.cpu_pods, "mismatches": mism},
    }))


if __name__ == "__main__":
    main()

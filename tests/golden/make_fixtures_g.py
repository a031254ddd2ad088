"""Seventh fixture batch: DefaultPreemption, transcribed by hand as data from
pkg/scheduler/framework/plugins/defaultpreemption/default_preemption_test.go:

  TestDryRunPreemption    :615   every case whose plugins are in-tree (NodeResourcesFit,
                                 InterPodAffinity, PodTopologySpread); the ones registering the fake
                                 FalseFilter / TrueFilter / MatchFilter plugins or a fake filter return
                                 code have no in-tree equivalent and are left out
  TestSelectBestCandidate :1375  all nine cases (DryRunPreemption over every node, SelectCandidate)
  TestPodEligibleToPreemptOthers :1961  all five cases (see eligible_cases)

Each case's profile enables exactly the plugins the test registers.  The test runs DryRunPreemption
over every node sorted by name ("allNodes": true; the nodes are added in name order, one nodeTree
zone, so snapshot order is name order); the random offset is the value the test's comments state for
rand.NewSource(4) (cycle 0 -> 4, 1 -> 1, 2 -> 3) where parallelism is disabled, 0 elsewhere (there
every node is checked, so the offset cannot change the candidate set).  Expected candidates compare
as the test compares them: victims sorted by name, candidates sorted by node name.

A case the device path declines would carry "device": "ENOTSUP" (none does).
Output: tests/golden/preemption.json (data only).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/framework/plugins/defaultpreemption/default_preemption_test.go"
ALL = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
       "PodTopologySpread", "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"]

NEG, LOW, MID, HIGH, VHIGH = -100, 0, 100, 1000, 10000  # :79
SMALL = {"cpu": "100m", "memory": "100"}                # :81-96
MEDIUM = {"cpu": "200m", "memory": "200"}
LARGE = {"cpu": "300m", "memory": "300"}
VLARGE = {"cpu": "500m", "memory": "500"}


def only(*keep):
    return {"disabledPlugins": [p for p in ALL if p not in keep]}


def epoch(ns):  # metav1.NewTime(time.Unix(0, ns)), :98-104
    return f"1970-01-01T00:00:00.{ns:09d}Z"


def node(spec):
    """st.MakeNode().Capacity(veryLargeRes) (wrappers.go:924-933: pods=32 added); a name "a/b/c"
    gives labels hostname=a, zone=b, region=c (:1251-1265)."""
    parts = spec.split("/")
    labels = dict(zip(["hostname", "zone", "region"], parts))
    res = dict(VLARGE, pods="32")
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": parts[0], "labels": labels},
            "spec": {}, "status": {"capacity": res, "allocatable": res}}


def pod(name, prio=None, node_name=None, req=None, start=None, labels=None, anti_exists=None, spreads=None,
        policy=None):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": "default", "uid": name, "labels": dict(labels or {})},
         "spec": {"containers": []}, "status": {}}
    if prio is not None:
        p["spec"]["priority"] = prio
    if policy:
        p["spec"]["preemptionPolicy"] = policy
    if node_name:
        p["spec"]["nodeName"] = node_name
    if req:
        p["spec"]["containers"].append({"name": "con0", "image": "pause", "resources": {"requests": dict(req)}})
    if start is not None:
        p["status"]["startTime"] = epoch(start)
    if anti_exists:  # PodAntiAffinityExists(key, topologyKey, Required)
        key, tk = anti_exists
        p["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchExpressions": [{"key": key, "operator": "Exists"}]}, "topologyKey": tk}]}}
    if spreads:
        p["spec"]["topologySpreadConstraints"] = spreads
    return p


def spread(skew, key):  # SpreadConstraint(skew, key, DoNotSchedule, Exists("foo"), ...)
    return {"maxSkew": skew, "topologyKey": key, "whenUnsatisfiable": "DoNotSchedule",
            "labelSelector": {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}}


def pdb(allowed, disrupted=()):
    return {"metadata": {}, "spec": {"selector": {"matchLabels": {"app": "foo"}}},
            "status": {"disruptionsAllowed": allowed, "disruptedPods": {n: "2020-01-01T00:00:00Z" for n in disrupted}}}


def cand(victims, viol=0):
    return {"victims": sorted(victims), "numPDBViolations": viol}


def dry_run(line, name, nodes, preemptor, init, expect, plugins=("NodeResourcesFit",), pdbs=(), args=None,
            offset=0, device=None):
    a = {"allNodes": True, "offset": offset, "pdbs": list(pdbs)}
    a.update(args or {})
    c = {"src": f"{SRC}:{line}", "name": f"DryRunPreemption: {name}", "kind": "preempt", "config": only(*plugins),
         "namespaces": [], "nodes": [node(n) for n in nodes], "existing": init, "pod": preemptor, "args": a,
         "expect": {"candidates": expect}}
    if device:
        c["device"] = device
    return c


def dry_run_cases():
    n2 = ["node1", "node2"]
    n5 = ["node1", "node2", "node3", "node4", "node5"]
    out = [
        dry_run(681, "a pod that fits on both nodes when lower priority pods are preempted", n2,
                pod("p", HIGH, req=LARGE), [pod("p1", MID, "node1", LARGE), pod("p2", MID, "node2", LARGE)],
                {"node1": cand(["p1"]), "node2": cand(["p2"])}),
        dry_run(712, "a pod that would fit on the nodes, but other pods running are higher priority", n2,
                pod("p", LOW, req=LARGE), [pod("p1", MID, "node1", LARGE), pod("p2", MID, "node2", LARGE)], {}),
        dry_run(728, "medium priority pod is preempted, but lower priority one stays as it is small", n2,
                pod("p", HIGH, req=LARGE),
                [pod("p1.1", LOW, "node1", SMALL), pod("p1.2", MID, "node1", LARGE), pod("p2", MID, "node2", LARGE)],
                {"node1": cand(["p1.2"]), "node2": cand(["p2"])}),
        dry_run(760, "mixed priority pods are preempted", n2, pod("p", HIGH, req=LARGE),
                [pod("p1.1", MID, "node1", SMALL), pod("p1.2", LOW, "node1", SMALL), pod("p1.3", MID, "node1", MEDIUM),
                 pod("p1.4", HIGH, "node1", SMALL), pod("p2", HIGH, "node2", LARGE)],
                {"node1": cand(["p1.2", "p1.3"])}),
        dry_run(791, "mixed priority pods are preempted, pick later StartTime one when priorities are equal", n2,
                pod("p", HIGH, req=LARGE),
                [pod("p1.1", LOW, "node1", SMALL, 5), pod("p1.2", LOW, "node1", SMALL, 4),
                 pod("p1.3", MID, "node1", MEDIUM, 3), pod("p1.4", HIGH, "node1", SMALL, 2),
                 pod("p2", HIGH, "node2", LARGE, 1)],
                {"node1": cand(["p1.1", "p1.3"])}),
        dry_run(822, "pod with anti-affinity is preempted", n2, pod("p", HIGH, req=SMALL, labels={"foo": ""}),
                [pod("p1.1", LOW, "node1", SMALL, labels={"foo": ""}, anti_exists=("foo", "hostname")),
                 pod("p1.2", MID, "node1", SMALL), pod("p1.3", HIGH, "node1", SMALL), pod("p2", HIGH, "node2", SMALL)],
                {"node1": cand(["p1.1"])}, plugins=("NodeResourcesFit", "InterPodAffinity")),
        dry_run(854, "preemption to resolve pod topology spread filter failure",
                ["node-a/zone1", "node-b/zone1", "node-x/zone2"],
                pod("p", HIGH, labels={"foo": ""}, spreads=[spread(1, "zone"), spread(1, "hostname")]),
                [pod("pod-a1", MID, "node-a", labels={"foo": ""}), pod("pod-a2", LOW, "node-a", labels={"foo": ""}),
                 pod("pod-b1", LOW, "node-b", labels={"foo": ""}), pod("pod-x1", HIGH, "node-x", labels={"foo": ""}),
                 pod("pod-x2", HIGH, "node-x", labels={"foo": ""})],
                {"node-a": cand(["pod-a2"]), "node-b": cand(["pod-b1"])}, plugins=("PodTopologySpread",)),
        dry_run(908, "preemption with violation of same pdb", ["node1"], pod("p", HIGH, req=VLARGE),
                [pod("p1.1", MID, "node1", MEDIUM, labels={"app": "foo"}),
                 pod("p1.2", MID, "node1", MEDIUM, labels={"app": "foo"})],
                {"node1": cand(["p1.1", "p1.2"], 1)}, pdbs=[pdb(1)]),
        dry_run(943, "pdb violation, the victim doesn't belong to DisruptedPods", ["node1"], pod("p", HIGH, req=VLARGE),
                [pod("p1.1", MID, "node1", MEDIUM, labels={"app": "foo"}),
                 pod("p1.2", MID, "node1", MEDIUM, labels={"app": "foo"})],
                {"node1": cand(["p1.1", "p1.2"], 1)}, pdbs=[pdb(1, ["p2"])]),
        dry_run(978, "pdb violation, the victim belongs to DisruptedPods", ["node1"], pod("p", HIGH, req=VLARGE),
                [pod("p1.1", MID, "node1", MEDIUM, labels={"app": "foo"}),
                 pod("p1.2", MID, "node1", MEDIUM, labels={"app": "foo"})],
                {"node1": cand(["p1.1", "p1.2"], 0)}, pdbs=[pdb(1, ["p1.2"])]),
        dry_run(1013, "pdb violation, the victim in DisruptedPods is treated as 'nonViolating'", ["node1"],
                pod("p", HIGH, req=VLARGE),
                [pod("p1.1", MID, "node1", MEDIUM, labels={"app": "foo"}),
                 pod("p1.2", MID, "node1", MEDIUM, labels={"app": "foo"}),
                 pod("p1.3", MID, "node1", MEDIUM, labels={"app": "foo"})],
                {"node1": cand(["p1.1", "p1.2", "p1.3"], 1)}, pdbs=[pdb(1, ["p1.3"])]),
        dry_run(1050, "all nodes are possible candidates, but DefaultPreemptionArgs limits to 2", n5,
                pod("p", HIGH, req=LARGE), [pod(f"p{i}", MID, f"node{i}", LARGE) for i in range(1, 6)],
                {"node1": cand(["p1"]), "node5": cand(["p5"])},
                args={"minCandidateNodesPercentage": 40, "minCandidateNodesAbsolute": 1}, offset=4),
        dry_run(1087, "some nodes are not possible candidates, DefaultPreemptionArgs limits to 2", n5,
                pod("p", HIGH, req=LARGE),
                [pod("p1", MID, "node1", LARGE), pod("p2", VHIGH, "node2", LARGE), pod("p3", MID, "node3", LARGE),
                 pod("p4", MID, "node4", LARGE), pod("p5", VHIGH, "node5", LARGE)],
                {"node1": cand(["p1"]), "node3": cand(["p3"])},
                args={"minCandidateNodesPercentage": 40, "minCandidateNodesAbsolute": 1}, offset=4),
        dry_run(1193, "preemption looks past numCandidates until a non-PDB violating node is found", n5,
                pod("p", HIGH, req=LARGE),
                [pod("p1", MID, "node1", LARGE, labels={"app": "foo"}), pod("p2", MID, "node2", LARGE, labels={"app": "foo"}),
                 pod("p3", MID, "node3", LARGE), pod("p4", MID, "node4", LARGE),
                 pod("p5", MID, "node5", LARGE, labels={"app": "foo"})],
                {"node1": cand(["p1"], 1), "node3": cand(["p3"]), "node5": cand(["p5"], 1)},
                args={"minCandidateNodesPercentage": 40, "minCandidateNodesAbsolute": 2}, pdbs=[pdb(0)], offset=4),
    ]
    # :1124 "preemption offset across multiple scheduling cycles and wrap around": three preemptors,
    # offsets 4, 1, 3 (one case per cycle; DryRunPreemption changes no state)
    init = [pod(f"p{i}", MID, f"node{i}", LARGE) for i in range(1, 6)]
    for k, (off, want) in enumerate(((4, ("node1", "node5")), (1, ("node2", "node3")), (3, ("node4", "node5")))):
        out.append(dry_run(1124, f"preemption offset across multiple scheduling cycles, cycle {k}", n5,
                           pod(f"tp{k + 1}", HIGH, req=LARGE), init,
                           {n: cand([f"p{n[-1]}"]) for n in want},
                           args={"minCandidateNodesPercentage": 40, "minCandidateNodesAbsolute": 1}, offset=off))
    return out


def best(line, name, nodes, preemptor, pods, expected):
    return {"src": f"{SRC}:{line}", "name": f"SelectBestCandidate: {name}", "kind": "preempt",
            "config": only("NodeResourcesFit"), "namespaces": [], "nodes": [node(n) for n in nodes],
            "existing": pods, "pod": preemptor, "args": {"allNodes": True, "offset": 0},
            "expect": {"selected_in": expected}}


def best_cases():
    n3 = ["node1", "node2", "node3"]
    P = lambda n, pr, nd, r, t=0: pod(n, pr, nd, r, t)  # noqa: E731
    return [
        best(1385, "a pod that fits on both nodes when lower priority pods are preempted", ["node1", "node2"],
             pod("p", HIGH, req=LARGE), [P("p1", MID, "node1", LARGE), P("p2", MID, "node2", LARGE)],
             ["node1", "node2"]),
        best(1396, "node with min highest priority pod is picked", n3, pod("p", HIGH, req=VLARGE),
             [P("p1.1", MID, "node1", MEDIUM), P("p1.2", MID, "node1", LARGE), P("p2.1", MID, "node2", MEDIUM),
              P("p2.2", LOW, "node2", MEDIUM), P("p3.1", LOW, "node3", MEDIUM), P("p3.2", LOW, "node3", MEDIUM)],
             ["node3"]),
        best(1411, "when highest priorities are the same, minimum sum of priorities is picked", n3,
             pod("p", HIGH, req=VLARGE),
             [P("p1.1", MID, "node1", MEDIUM), P("p1.2", MID, "node1", LARGE), P("p2.1", MID, "node2", LARGE),
              P("p2.2", LOW, "node2", MEDIUM), P("p3.1", MID, "node3", MEDIUM), P("p3.2", MID, "node3", MEDIUM)],
             ["node2"]),
        best(1426, "when highest priority and sum are the same, minimum number of pods is picked", n3,
             pod("p", HIGH, req=VLARGE),
             [P("p1.1", MID, "node1", SMALL), P("p1.2", NEG, "node1", SMALL), P("p1.3", MID, "node1", SMALL),
              P("p1.4", NEG, "node1", SMALL), P("p2.1", MID, "node2", LARGE), P("p2.2", NEG, "node2", MEDIUM),
              P("p3.1", MID, "node3", MEDIUM), P("p3.2", NEG, "node3", SMALL), P("p3.3", LOW, "node3", SMALL)],
             ["node2"]),
        best(1446, "sum of adjusted priorities is considered", n3, pod("p", HIGH, req=VLARGE),
             [P("p1.1", MID, "node1", SMALL), P("p1.2", NEG, "node1", SMALL), P("p1.3", NEG, "node1", SMALL),
              P("p2.1", MID, "node2", LARGE), P("p2.2", NEG, "node2", MEDIUM), P("p3.1", MID, "node3", MEDIUM),
              P("p3.2", NEG, "node3", SMALL), P("p3.3", LOW, "node3", SMALL)],
             ["node2"]),
        best(1463, "non-overlapping lowest high priority, sum priorities, and number of pods",
             ["node1", "node2", "node3", "node4"], pod("p", VHIGH, req=VLARGE),
             [P("p1.1", MID, "node1", SMALL), P("p1.2", LOW, "node1", SMALL), P("p1.3", LOW, "node1", SMALL),
              P("p2.1", HIGH, "node2", LARGE), P("p3.1", MID, "node3", MEDIUM), P("p3.2", LOW, "node3", SMALL),
              P("p3.3", LOW, "node3", SMALL), P("p3.4", LOW, "node3", MEDIUM), P("p4.1", MID, "node4", MEDIUM),
              P("p4.2", MID, "node4", SMALL), P("p4.3", MID, "node4", SMALL), P("p4.4", NEG, "node4", SMALL)],
             ["node1"]),
        best(1484, "same priority, same number of victims, different start time for each node's pod", n3,
             pod("p", HIGH, req=VLARGE),
             [P("p1.1", MID, "node1", MEDIUM, 2), P("p1.2", MID, "node1", MEDIUM, 2), P("p2.1", MID, "node2", MEDIUM, 3),
              P("p2.2", MID, "node2", MEDIUM, 3), P("p3.1", MID, "node3", MEDIUM, 1), P("p3.2", MID, "node3", MEDIUM, 1)],
             ["node2"]),
        best(1499, "same priority, same number of victims, different start time for all pods", n3,
             pod("p", HIGH, req=VLARGE),
             [P("p1.1", MID, "node1", MEDIUM, 4), P("p1.2", MID, "node1", MEDIUM, 2), P("p2.1", MID, "node2", MEDIUM, 5),
              P("p2.2", MID, "node2", MEDIUM, 1), P("p3.1", MID, "node3", MEDIUM, 3), P("p3.2", MID, "node3", MEDIUM, 6)],
             ["node3"]),
        best(1514, "different priority, same number of victims, different start time for all pods", n3,
             pod("p", HIGH, req=VLARGE),
             [P("p1.1", LOW, "node1", MEDIUM, 4), P("p1.2", MID, "node1", MEDIUM, 2), P("p2.1", MID, "node2", MEDIUM, 6),
              P("p2.2", LOW, "node2", MEDIUM, 1), P("p3.1", LOW, "node3", MEDIUM, 3), P("p3.2", MID, "node3", MEDIUM, 5)],
             ["node2"]),
    ]


def eligible_cases():
    """TestPodEligibleToPreemptOthers :1961.  The nominated node's status is the failed cycle's: the
    first case's UnschedulableAndUnresolvable comes from an untolerated taint (TaintToleration on),
    the others' nil status from a profile with no filter plugin.  "Eligible" shows as the dry run
    going ahead (no candidate here: KSG_PREEMPT_NO_CANDIDATES = 2); not eligible is reason 1."""
    def term(p, condition=False):
        p["metadata"]["deletionTimestamp"] = "2020-01-01T00:00:00Z"
        if condition:
            p["status"]["conditions"] = [{"type": "DisruptionTarget", "status": "True", "reason": "PreemptionByScheduler"}]
        return p

    def nominated(p):
        p["status"]["nominatedNodeName"] = "node1"
        return p

    bare = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "node1"}, "spec": {}, "status": {}}
    tainted = json.loads(json.dumps(bare))
    tainted["spec"]["taints"] = [{"key": "k", "value": "v", "effect": "NoSchedule"}]

    def case(line, name, nodes, pods, p, reason, cfg=None):
        return {"src": f"{SRC}:{line}", "name": f"PodEligibleToPreemptOthers: {name}", "kind": "preempt",
                "config": cfg or only(), "namespaces": [], "nodes": nodes, "existing": pods, "pod": p, "args": {},
                "expect": {"reason": reason, "candidates": {}}}
    return [
        case(1971, "Pod with nominated node (status UnschedulableAndUnresolvable)", [tainted],
             [term(pod("p1", LOW, "node1"))], nominated(pod("p_with_nominated_node", HIGH)), 2,
             only("TaintToleration")),
        case(1979, "Pod without nominated node", [], [], pod("p_without_nominated_node", HIGH), 2),
        case(1987, "Pod with 'PreemptNever' preemption policy", [], [],
             pod("p_with_preempt_never_policy", HIGH, policy="Never"), 1),
        case(1995, "preemption victim pod terminating, as indicated by the DisruptionTarget condition", [bare],
             [term(pod("p1", LOW, "node1"), True)], nominated(pod("p_with_nominated_node", HIGH)), 1),
        case(2003, "non-victim Pods terminating", [bare], [term(pod("p1", LOW, "node1"))],
             nominated(pod("p_with_nominated_node", HIGH)), 2),
    ]


def cases():
    return dry_run_cases() + best_cases() + eligible_cases()


if __name__ == "__main__":
    with open(os.path.join(HERE, "preemption.json"), "w") as f:
        json.dump({"source": "make_fixtures_g.py", "cases": cases()}, f, indent=1)
        f.write("\n")

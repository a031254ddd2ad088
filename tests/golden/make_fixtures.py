"""Regenerates tests/golden/*.json: golden vectors transcribed (as data) from the
reference's own table-driven unit tests.  Each case names the Go test file:line it
comes from; the expected values are copied verbatim from those tables.

Cluster objects are re-expressed in the v1 JSON schema through ksg.objects (the
analogue of st.MakePod()/st.MakeNode()).  Nothing here imports or runs the reference;
the Go sources were read as text.  Run:  python tests/golden/make_fixtures.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "kubernetes-kubernetes_amd"))
from ksg.objects import NodeW, PodW, expr, make_namespace  # noqa: E402

U, UU, SKIP, ERR = 2, 3, 5, 1
MB = 1024 * 1024
_uid = [0]


def pod(name="p", ns="default"):
    _uid[0] += 1
    return PodW(name, ns, uid=f"uid-{_uid[0]}")


def st_node(name, cap=None):
    """st.MakeNode().Name(n).Capacity(cap): pods=32 is added by Capacity (wrappers.go:924-933)."""
    n = NodeW(name)
    if cap is not None:
        res = {"pods": "32"}
        res.update(cap)
        n.capacity(res)
    return n


def make_node(name, milli_cpu, memory, ext=None):
    """noderesources/util_test.go:43-57 makeNode (no pods allocatable)."""
    res = {"cpu": f"{milli_cpu}m", "memory": str(memory)}
    for k, v in (ext or {}).items():
        res[k] = str(v)
    return NodeW(name).capacity(res)


def score_case(src, name, nodes, pod_obj, plugin, expect, existing=(), config=None, norm=True, status=0,
               namespaces=()):
    return {"src": src, "name": name, "kind": "score", "plugin": plugin, "config": config or {},
            "namespaces": list(namespaces), "nodes": [n.obj() if hasattr(n, "obj") else n for n in nodes],
            "existing": [p.obj() if hasattr(p, "obj") else p for p in existing],
            "pod": pod_obj.obj() if hasattr(pod_obj, "obj") else pod_obj,
            "expect": {"status": status, ("normalized" if norm else "raw"): expect}}


def filter_case(src, name, nodes, pod_obj, plugin, codes, existing=(), config=None, prefilter=0, reasons=None,
                namespaces=()):
    e = {"prefilter": prefilter, "codes": codes}
    if reasons is not None:
        e["reasons"] = reasons
    return {"src": src, "name": name, "kind": "filter", "plugin": plugin, "config": config or {},
            "namespaces": list(namespaces), "nodes": [n.obj() if hasattr(n, "obj") else n for n in nodes],
            "existing": [p.obj() if hasattr(p, "obj") else p for p in existing],
            "pod": pod_obj.obj() if hasattr(pod_obj, "obj") else pod_obj, "expect": e}


def config_error_case(src, name, config):
    return {"src": src, "name": name, "kind": "config_error", "config": config}


# ---------------------------------------------------------------------------------------
# helper/normalize_score_test.go:27-73 (DefaultNormalizeScore), driven through the two
# plugins that use it: NodeAffinity (reverse=false) and TaintToleration (reverse=true).
# ---------------------------------------------------------------------------------------
def normalize_cases():
    src = "pkg/scheduler/framework/plugins/helper/normalize_score_test.go:27-73"
    vectors = [
        (False, [1, 2, 3, 4], [25, 50, 75, 100]),
        (True, [1, 2, 3, 4], [75, 50, 25, 0]),
        (False, [1000, 10, 20, 30], [100, 1, 2, 3]),
        (True, [1000, 10, 20, 30], [0, 99, 98, 97]),
        (False, [1, 1, 1, 1], [100, 100, 100, 100]),
        (False, [1000, 1, 1, 1], [100, 0, 0, 0]),
        (True, [0, 1, 1, 1], [100, 0, 0, 0]),
        (False, [0, 0, 0, 0], [0, 0, 0, 0]),
        (True, [0, 0, 0, 0], [100, 100, 100, 100]),
    ]
    out = []
    for ci, (reverse, raw, want) in enumerate(vectors):
        nodes = []
        if reverse:
            # raw = number of PreferNoSchedule taints the pod does not tolerate
            for i, r in enumerate(raw):
                nodes.append(NodeW(f"n{i}").taints([{"key": f"t{k}", "value": "v", "effect": "PreferNoSchedule"}
                                                    for k in range(r)]))
            p = pod()
            out.append(score_case(src, f"case_{ci}_reverse", nodes, p, "TaintToleration", want))
        else:
            # raw = sum of weights of matching preferred terms (weights <= 100 each)
            terms = []
            for i, r in enumerate(raw):
                nodes.append(NodeW(f"n{i}").label("idx", f"v{i}"))
                left = r
                while left > 0:
                    w = min(100, left)
                    terms.append((w, {"matchExpressions": [expr("idx", "In", [f"v{i}"])]}))
                    left -= w
            p = pod()
            if terms:
                p.node_affinity_preferred(terms)
            else:  # keep the plugin active with a term that matches nothing
                p.node_affinity_preferred([(1, {"matchExpressions": [expr("idx", "In", ["none"])]})])
            out.append(score_case(src, f"case_{ci}", nodes, p, "NodeAffinity", want))
    return out


# ---------------------------------------------------------------------------------------
# noderesources/least_allocated_test.go:38-439
# ---------------------------------------------------------------------------------------
def least_allocated_cases():
    src = "pkg/scheduler/framework/plugins/noderesources/least_allocated_test.go"
    default = [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]
    ext = "abc.com/xyz"
    extset = default + [{"name": ext, "weight": 1}]

    def cfg(res):
        return {"nodeResourcesFit": {"scoringStrategy": {"type": "LeastAllocated", "resources": res}}}

    two = lambda: [  # noqa: E731
        st_node("node1", {"cpu": "4000", "memory": "10000"}), st_node("node2", {"cpu": "4000", "memory": "10000"})]
    req2 = lambda p: p.req({"cpu": "1000", "memory": "2000"}).req({"cpu": "2000", "memory": "3000"})  # noqa: E731
    C = []
    C.append(score_case(src + ":61", "nothing scheduled, nothing requested", two(), pod(), "NodeResourcesFit",
                        [100, 100], config=cfg(default), norm=False))
    C.append(score_case(src + ":72", "nothing scheduled, resources requested, differently sized nodes",
                        [st_node("node1", {"cpu": "4000", "memory": "10000"}),
                         st_node("node2", {"cpu": "6000", "memory": "10000"})],
                        req2(pod()), "NodeResourcesFit", [37, 50], config=cfg(default), norm=False))
    C.append(score_case(src + ":86", "Resources not set, pods scheduled with error",
                        [st_node("node1", {"cpu": "4000", "memory": "10000"}),
                         st_node("node2", {"cpu": "6000", "memory": "10000"})],
                        req2(pod()), "NodeResourcesFit", [0, 0], config=cfg([]), norm=False, status=ERR))
    C.append(score_case(src + ":101", "no resources requested, pods scheduled", two(), pod(), "NodeResourcesFit",
                        [100, 100], existing=[pod().node("node1"), pod().node("node1"), pod().node("node2"),
                                              pod().node("node2")], config=cfg(default), norm=False))
    C.append(score_case(src + ":116", "no resources requested, pods scheduled with resources",
                        [st_node("node1", {"cpu": "10000", "memory": "20000"}),
                         st_node("node2", {"cpu": "10000", "memory": "20000"})], pod(), "NodeResourcesFit", [70, 57],
                        existing=[pod().node("node1").req({"cpu": "3000", "memory": "0"}),
                                  pod().node("node1").req({"cpu": "3000", "memory": "0"}),
                                  pod().node("node2").req({"cpu": "3000", "memory": "0"}),
                                  pod().node("node2").req({"cpu": "3000", "memory": "5000"})],
                        config=cfg(default), norm=False))
    C.append(score_case(src + ":131", "resources requested, pods scheduled with resources",
                        [st_node("node1", {"cpu": "10000", "memory": "20000"}),
                         st_node("node2", {"cpu": "10000", "memory": "20000"})], req2(pod()), "NodeResourcesFit",
                        [57, 45], existing=[pod().node("node1").req({"cpu": "3000", "memory": "0"}),
                                            pod().node("node2").req({"cpu": "3000", "memory": "5000"})],
                        config=cfg(default), norm=False))
    C.append(score_case(src + ":148", "resources requested, pods scheduled with resources, differently sized nodes",
                        [st_node("node1", {"cpu": "10000", "memory": "20000"}),
                         st_node("node2", {"cpu": "10000", "memory": "50000"})], req2(pod()), "NodeResourcesFit",
                        [57, 60], existing=[pod().node("node1").req({"cpu": "3000", "memory": "0"}),
                                            pod().node("node2").req({"cpu": "3000", "memory": "5000"})],
                        config=cfg(default), norm=False))
    C.append(score_case(src + ":165", "requested resources exceed node capacity", two(),
                        pod().req({"cpu": "3000", "memory": "0"}), "NodeResourcesFit", [50, 25],
                        existing=[pod().node("node1").req({"cpu": "3000", "memory": "0"}),
                                  pod().node("node2").req({"cpu": "3000", "memory": "5000"})],
                        config=cfg(default), norm=False))
    C.append(score_case(src + ":178", "zero node resources, pods scheduled with resources",
                        [NodeW("node1"), NodeW("node2")], pod(), "NodeResourcesFit", [0, 0],
                        existing=[pod().node("node1").req({"cpu": "3000", "memory": "0"}),
                                  pod().node("node2").req({"cpu": "3000", "memory": "5000"})],
                        config=cfg(default), norm=False))
    C.append(score_case(src + ":191", "different weight on CPU and memory, differently sized nodes",
                        [st_node("node1", {"cpu": "4000", "memory": "10000"}),
                         st_node("node2", {"cpu": "6000", "memory": "10000"})], req2(pod().node("node1")),
                        "NodeResourcesFit", [41, 50],
                        config=cfg([{"name": "memory", "weight": 2}, {"name": "cpu", "weight": 1}]), norm=False))
    C.append(config_error_case(src + ":208", "resource with negative weight",
                               cfg([{"name": "memory", "weight": -1}, {"name": "cpu", "weight": 1}])))
    C.append(config_error_case(src + ":248", "resource weight larger than MaxNodeScore",
                               cfg([{"name": "memory", "weight": 1}, {"name": "cpu", "weight": 101}])))
    C.append(score_case(src + ":268", "bypass extended resource if the pod does not request",
                        [st_node("node1", {"cpu": "6000", "memory": "10000"}),
                         st_node("node2", {"cpu": "6000", "memory": "10000", ext: "4"})], req2(pod().node("node1")),
                        "NodeResourcesFit", [50, 50], config=cfg(extset), norm=False))
    C.append(score_case(src + ":281", "honor extended resource if the pod requests",
                        [st_node("node1", {"cpu": "6000", "memory": "10000", ext: "4"}),
                         st_node("node2", {"cpu": "6000", "memory": "10000", ext: "10"})],
                        pod().node("node1").req({"cpu": "3000", "memory": "5000", ext: "2"}),
                        "NodeResourcesFit", [50, 60], config=cfg(extset), norm=False))
    C.append(score_case(src + ":294", "if the node doesn't have a resource",
                        [st_node("node1", {"cpu": "6000", "memory": "10000"}),
                         st_node("node2", {"cpu": "6000", "memory": "10000", ext: "4"})],
                        pod().node("node1").req({"cpu": "3000", "memory": "4000"}), "NodeResourcesFit", [55, 55],
                        config=cfg([{"name": ext, "weight": 2}, {"name": "cpu", "weight": 1},
                                    {"name": "memory", "weight": 1}]), norm=False))
    return C


# ---------------------------------------------------------------------------------------
# noderesources/balanced_allocation_test.go:41-316
# ---------------------------------------------------------------------------------------
def balanced_cases():
    src = "pkg/scheduler/framework/plugins/noderesources/balanced_allocation_test.go"
    default = {"balancedAllocation": {"resources": [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]}}
    gpu3 = {"balancedAllocation": {"resources": [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1},
                                                 {"name": "nvidia.com/gpu", "weight": 1}]}}
    cm = lambda c, m: {"cpu": c, "memory": m}  # noqa: E731
    B = "NodeResourcesBalancedAllocation"
    C = []
    C.append(score_case(src + ":63", "nothing scheduled, nothing requested, skip in PreScore",
                        [make_node("node1", 4000, 10000), make_node("node2", 4000, 10000)], pod(), B, [0, 0],
                        config=default, norm=False, status=SKIP))
    C.append(score_case(src + ":79", "nothing scheduled, resources requested, differently sized nodes",
                        [make_node("node1", 4000, 10000), make_node("node2", 6000, 10000)],
                        pod().req(cm("1000m", "2000")).req(cm("2000m", "3000")), B, [68, 75], config=default,
                        norm=False))
    C.append(score_case(src + ":97", "resources requested, pods scheduled with resources",
                        [make_node("node1", 10000, 20000), make_node("node2", 10000, 20000)],
                        pod().req(cm("1000m", "2000")).req(cm("2000m", "3000")), B, [73, 74],
                        existing=[pod().node("node1").req({"cpu": "1000m"}).req({"cpu": "2000m"}),
                                  pod().node("node2").req(cm("1000m", "2000")).req(cm("2000m", "3000"))],
                        config=default, norm=False))
    C.append(score_case(src + ":120", "pods scheduled with resources, differently sized nodes",
                        [make_node("node1", 10000, 20000), make_node("node2", 10000, 50000)],
                        pod().req(cm("1000m", "2000")).req(cm("2000m", "3000")), B, [73, 70],
                        existing=[pod().node("node1").req({"cpu": "1000m"}).req({"cpu": "2000m"}),
                                  pod().node("node2").req(cm("1000m", "2000")).req(cm("2000m", "3000"))],
                        config=default, norm=False))
    C.append(score_case(src + ":143", "nodes to reach min/max score",
                        [make_node("node1", 3000, 5000), make_node("node2", 3000, 5000)],
                        pod().req({"memory": "2000"}).req({"memory": "3000"}), B, [100, 50],
                        existing=[pod().node("node1").req({"cpu": "1000m"}).req({"cpu": "2000m"})],
                        config=default, norm=False))
    C.append(score_case(src + ":165", "requested resources at node capacity",
                        [make_node("node1", 6000, 10000), make_node("node2", 6000, 10000)],
                        pod().req({"cpu": "1000m"}).req({"cpu": "2000m"}), B, [62, 62],
                        existing=[pod().node("node1").req({"cpu": "1000m"}).req({"cpu": "2000m"}),
                                  pod().node("node2").req(cm("1000m", "2000")).req(cm("2000m", "3000"))],
                        config=default, norm=False))
    C.append(score_case(src + ":190", "scalar resource is included if pod requests it",
                        [make_node("node1", 3500, 40000, {"nvidia.com/gpu": 8}),
                         make_node("node2", 3500, 40000, {"nvidia.com/gpu": 8})],
                        pod().req({"cpu": "0", "memory": "0", "nvidia.com/gpu": "1"}), B, [75, 76],
                        existing=[pod().node("node1").req(cm("1000m", "2000")).req(
                            {"cpu": "2000m", "memory": "3000", "nvidia.com/gpu": "3"}),
                            pod().node("node2").req(cm("1000m", "2000")).req(cm("2000m", "3000"))],
                        config=gpu3, norm=False))
    C.append(score_case(src + ":218", "scalar resource is not included if pod doesn't request it",
                        [make_node("node1", 3500, 40000, {"nvidia.com/gpu": 8}), make_node("node2", 3500, 40000)],
                        pod().req(cm("1000m", "2000")).req(cm("2000m", "3000")), B, [56, 56], config=gpu3,
                        norm=False))
    return C


# ---------------------------------------------------------------------------------------
# tainttoleration/taint_toleration_test.go:57-328 (score) and :329-520 (filter)
# ---------------------------------------------------------------------------------------
def taint_cases():
    src = "pkg/scheduler/framework/plugins/tainttoleration/taint_toleration_test.go"
    T = "TaintToleration"
    tn = lambda n, ts: NodeW(n).taints(ts)  # noqa: E731
    tp = lambda ts: pod("pod1").tolerations(ts)  # noqa: E731
    PNS, NS = "PreferNoSchedule", "NoSchedule"
    gate = {"featureGates": {"TaintTolerationComparisonOperators": True}}
    C = []
    C.append(score_case(src + ":67", "tolerated taints score higher", [
        tn("nodeA", [{"key": "foo", "value": "bar", "effect": PNS}]),
        tn("nodeB", [{"key": "foo", "value": "blah", "effect": PNS}])],
        tp([{"key": "foo", "operator": "Equal", "value": "bar", "effect": PNS}]), T, [100, 0]))
    both = [{"key": "cpu-type", "value": "arm64", "effect": PNS}, {"key": "disk-type", "value": "ssd", "effect": PNS}]
    C.append(score_case(src + ":90", "count of tolerated taints does not matter", [
        tn("nodeA", []), tn("nodeB", both[:1]), tn("nodeC", both)],
        tp([{"key": "cpu-type", "operator": "Equal", "value": "arm64", "effect": PNS},
            {"key": "disk-type", "operator": "Equal", "value": "ssd", "effect": PNS}]), T, [100, 100, 100]))
    C.append(score_case(src + ":129", "more intolerable taints, lower score", [
        tn("nodeA", []), tn("nodeB", both[:1]), tn("nodeC", both)],
        tp([{"key": "foo", "operator": "Equal", "value": "bar", "effect": PNS}]), T, [100, 50, 0]))
    C.append(score_case(src + ":161", "only PreferNoSchedule taints/tolerations are checked", [
        tn("nodeA", []), tn("nodeB", [{"key": "cpu-type", "value": "arm64", "effect": NS}]), tn("nodeC", both)],
        tp([{"key": "cpu-type", "operator": "Equal", "value": "arm64", "effect": NS},
            {"key": "disk-type", "operator": "Equal", "value": "ssd", "effect": NS}]), T, [100, 100, 0]))
    C.append(score_case(src + ":201", "no taints and tolerations", [
        tn("nodeA", []), tn("nodeB", both[:1])], tp([]), T, [100, 0]))
    C.append(score_case(src + ":218", "numeric Gt operator", [
        tn("nodeA", [{"key": "node.kubernetes.io/sla", "value": "800", "effect": PNS}]),
        tn("nodeB", [{"key": "node.kubernetes.io/sla", "value": "999", "effect": PNS}])],
        tp([{"key": "node.kubernetes.io/sla", "operator": "Gt", "value": "950", "effect": PNS}]), T, [0, 100],
        config=gate))
    C.append(score_case(src + ":240", "numeric Lt operator", [
        tn("nodeA", [{"key": "node.kubernetes.io/sla", "value": "950", "effect": PNS}]),
        tn("nodeB", [{"key": "node.kubernetes.io/sla", "value": "700", "effect": PNS}])],
        tp([{"key": "node.kubernetes.io/sla", "operator": "Lt", "value": "800", "effect": PNS}]), T, [0, 100],
        config=gate))
    # ---- filter (one node per case)
    fl = [
        ("no tolerations vs NoSchedule taint", [], [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], UU, None),
        ("dedicated user1 tolerated", [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}],
         [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], 0, None),
        ("user2 toleration vs user1 taint", [{"key": "dedicated", "operator": "Equal", "value": "user2", "effect": "NoSchedule"}],
         [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], UU, None),
        ("Exists toleration", [{"key": "foo", "operator": "Exists", "effect": "NoSchedule"}],
         [{"key": "foo", "value": "bar", "effect": "NoSchedule"}], 0, None),
        ("multiple tolerations and taints all tolerated",
         [{"key": "dedicated", "operator": "Equal", "value": "user2", "effect": "NoSchedule"},
          {"key": "foo", "operator": "Exists", "effect": "NoSchedule"}],
         [{"key": "dedicated", "value": "user2", "effect": "NoSchedule"}, {"key": "foo", "value": "bar", "effect": "NoSchedule"}],
         0, None),
        ("effect mismatch", [{"key": "foo", "operator": "Equal", "value": "bar", "effect": "PreferNoSchedule"}],
         [{"key": "foo", "value": "bar", "effect": "NoSchedule"}], UU, None),
        ("empty toleration effect matches all", [{"key": "foo", "operator": "Equal", "value": "bar"}],
         [{"key": "foo", "value": "bar", "effect": "NoSchedule"}], 0, None),
        ("PreferNoSchedule taint never filters", [{"key": "dedicated", "operator": "Equal", "value": "user2", "effect": "NoSchedule"}],
         [{"key": "dedicated", "value": "user1", "effect": "PreferNoSchedule"}], 0, None),
        ("no toleration, PreferNoSchedule taint", [], [{"key": "dedicated", "value": "user1", "effect": "PreferNoSchedule"}], 0, None),
        ("Gt below threshold", [{"key": "node.example.com/priority-level", "operator": "Gt", "value": "950", "effect": "NoSchedule"}],
         [{"key": "node.example.com/priority-level", "value": "800", "effect": "NoSchedule"}], UU, True),
        ("Gt above threshold", [{"key": "node.kubernetes.io/sla", "operator": "Gt", "value": "750", "effect": "NoSchedule"}],
         [{"key": "node.kubernetes.io/sla", "value": "950", "effect": "NoSchedule"}], 0, True),
        ("Lt above threshold", [{"key": "node.example.com/priority-level", "operator": "Lt", "value": "800", "effect": "NoSchedule"}],
         [{"key": "node.example.com/priority-level", "value": "950", "effect": "NoSchedule"}], UU, True),
        ("Lt below threshold", [{"key": "node.kubernetes.io/sla", "operator": "Lt", "value": "950", "effect": "NoSchedule"}],
         [{"key": "node.kubernetes.io/sla", "value": "800", "effect": "NoSchedule"}], 0, True),
        ("Gt vs non-numeric taint", [{"key": "node.kubernetes.io/sla", "operator": "Gt", "value": "950", "effect": "NoSchedule"}],
         [{"key": "node.kubernetes.io/sla", "value": "high", "effect": "NoSchedule"}], UU, True),
        # TestTaintTolerationFilterWithFeatureGate (:514-...)
        ("gate off: Gt toleration ignored", [{"key": "node.kubernetes.io/sla", "operator": "Gt", "value": "750", "effect": "NoSchedule"}],
         [{"key": "node.kubernetes.io/sla", "value": "950", "effect": "NoSchedule"}], UU, False),
        ("gate off: Lt toleration ignored", [{"key": "node.kubernetes.io/sla", "operator": "Lt", "value": "950", "effect": "NoSchedule"}],
         [{"key": "node.kubernetes.io/sla", "value": "800", "effect": "NoSchedule"}], UU, False),
        ("gate off: mixed, only Equal honored",
         [{"key": "dedicated", "operator": "Equal", "value": "user1", "effect": "NoSchedule"},
          {"key": "node.kubernetes.io/sla", "operator": "Gt", "value": "750", "effect": "NoSchedule"}],
         [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}], 0, False),
        ("gate off: mixed, Gt needed",
         [{"key": "dedicated", "operator": "Equal", "value": "user1", "effect": "NoSchedule"},
          {"key": "node.kubernetes.io/sla", "operator": "Gt", "value": "750", "effect": "NoSchedule"}],
         [{"key": "dedicated", "value": "user1", "effect": "NoSchedule"}, {"key": "node.kubernetes.io/sla", "value": "950", "effect": "NoSchedule"}],
         UU, False),
    ]
    for name, tols, taints, code, g in fl:
        C.append(filter_case(src + ":329", name, [tn("nodeA", taints)], tp(tols), T, [code],
                             config=gate if g else {}, reasons=[4 if code else 0]))
    return C


# ---------------------------------------------------------------------------------------
# nodeaffinity/node_affinity_test.go:41-935 (TestNodeAffinity: PreFilter + Filter)
# ---------------------------------------------------------------------------------------
def node_affinity_filter_cases():
    src = "pkg/scheduler/framework/plugins/nodeaffinity/node_affinity_test.go"
    NA = "NodeAffinity"
    C = []

    def case(name, p, labels=None, node_name="node1", code=0, prefilter=0, config=None, reason=None):
        n = NodeW(node_name)
        for k, v in (labels or {}).items():
            n.label(k, v)
        if reason is None:
            reason = 0 if code == 0 else 8  # KSG_R_NODE_AFFINITY_POD
        C.append(filter_case(src + ":41", name, [n], p, NA, [code], config=config, prefilter=prefilter,
                             reasons=None if prefilter else [reason]))

    req = lambda terms: pod().node_affinity_required(terms)  # noqa: E731
    case("missing labels", pod().node_selector({"foo": "bar"}), code=UU)
    case("same labels", pod().node_selector({"foo": "bar"}), {"foo": "bar"})
    case("node labels are superset", pod().node_selector({"foo": "bar"}), {"foo": "bar", "baz": "blah"})
    case("node labels are subset", pod().node_selector({"foo": "bar", "baz": "blah"}), {"foo": "bar"}, code=UU)
    case("In operator matches", req([{"matchExpressions": [expr("foo", "In", ["bar", "value2"])]}]), {"foo": "bar"})
    case("Gt operator matches", req([{"matchExpressions": [expr("kernel-version", "Gt", ["0204"])]}]),
         {"kernel-version": "0206"})
    case("NotIn operator matches", req([{"matchExpressions": [expr("mem-type", "NotIn", ["DDR", "DDR2"])]}]),
         {"mem-type": "DDR3"})
    case("Exists operator matches", req([{"matchExpressions": [expr("GPU", "Exists")]}]), {"GPU": "NVIDIA-GRID-K1"})
    case("affinity doesn't match labels", req([{"matchExpressions": [expr("foo", "In", ["value1", "value2"])]}]),
         {"foo": "bar"}, code=UU)
    case("empty MatchExpressions matches nothing", req([{"matchExpressions": []}]), {"foo": "bar"}, code=UU)
    case("no Affinity", pod(), {"foo": "bar"}, prefilter=SKIP)
    p = pod()
    p.o["spec"]["affinity"] = {"nodeAffinity": {}}
    case("Affinity but nil NodeSelector", p, {"foo": "bar"}, prefilter=SKIP)
    case("multiple matchExpressions ANDed match",
         req([{"matchExpressions": [expr("GPU", "Exists"), expr("GPU", "NotIn", ["AMD", "INTER"])]}]),
         {"GPU": "NVIDIA-GRID-K1"})
    case("multiple matchExpressions ANDed don't match",
         req([{"matchExpressions": [expr("GPU", "Exists"), expr("GPU", "In", ["AMD", "INTER"])]}]),
         {"GPU": "NVIDIA-GRID-K1"}, code=UU)
    case("multiple terms ORed", req([{"matchExpressions": [expr("foo", "In", ["bar", "value2"])]},
                                     {"matchExpressions": [expr("diffkey", "In", ["wrong", "value2"])]}]),
         {"foo": "bar"})
    case("Affinity and NodeSelector both satisfied",
         req([{"matchExpressions": [expr("foo", "Exists")]}]).node_selector({"foo": "bar"}), {"foo": "bar"})
    case("Affinity matches but NodeSelector not",
         req([{"matchExpressions": [expr("foo", "Exists")]}]).node_selector({"foo": "bar"}), {"foo": "barrrrrr"},
         code=UU)
    case("invalid value in Affinity term",
         req([{"matchExpressions": [expr("foo", "NotIn", ["invalid value: ___@#$%^"])]}]), {"foo": "bar"}, code=UU)
    mf = lambda vals: {"key": "metadata.name", "operator": "In", "values": vals}  # noqa: E731
    case("matchFields In matches", req([{"matchFields": [mf(["node1"])]}]), node_name="node1")
    case("matchFields In does not match", req([{"matchFields": [mf(["node1"])]}]), node_name="node2", code=UU)
    case("two terms: fields don't match, expressions match",
         req([{"matchFields": [mf(["node1"]), mf(["node2"])]},
              {"matchExpressions": [expr("foo", "In", ["bar"])]}]), {"foo": "bar"}, node_name="node2")
    case("one term: fields don't match, expressions match",
         req([{"matchFields": [mf(["node1"])], "matchExpressions": [expr("foo", "In", ["bar"])]}]), {"foo": "bar"},
         node_name="node2", code=UU)
    case("one term: both match",
         req([{"matchFields": [mf(["node1"])], "matchExpressions": [expr("foo", "In", ["bar"])]}]), {"foo": "bar"},
         node_name="node1")
    case("two terms: neither matches",
         req([{"matchFields": [mf(["node1"])]}, {"matchExpressions": [expr("foo", "In", ["not-match-to-bar"])]}]),
         {"foo": "bar"}, node_name="node2", code=UU)
    case("two terms of node.Name affinity", req([{"matchFields": [mf(["node1"])]}, {"matchFields": [mf(["node2"])]}]),
         node_name="node2")
    case("two conflicting matchField requirements", req([{"matchFields": [mf(["node1"]), mf(["node2"])]}]),
         {"foo": "bar"}, node_name="node2", code=UU, prefilter=UU)
    added = lambda terms: {"nodeAffinity": {"addedAffinity": {  # noqa: E731
        "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": terms}}}}
    case("matches added affinity and pod's", req([{"matchExpressions": [expr("zone", "In", ["foo"])]}]),
         {"zone": "foo"}, node_name="node2", config=added([{"matchFields": [mf(["node2"])]}]))
    case("matches added affinity but not pod's", req([{"matchExpressions": [expr("zone", "In", ["bar"])]}]),
         {"zone": "foo"}, node_name="node2", config=added([{"matchFields": [mf(["node2"])]}]), code=UU)
    case("doesn't match added affinity", pod(), {"zone": "foo"}, node_name="node2",
         config=added([{"matchExpressions": [expr("zone", "In", ["bar"])]}]), code=UU, reason=16)
    return C


# ---------------------------------------------------------------------------------------
# imagelocality/image_locality_test.go:36-420
# ---------------------------------------------------------------------------------------
def image_locality_cases():
    src = "pkg/scheduler/framework/plugins/imagelocality/image_locality_test.go"
    IL = "ImageLocality"

    def node(name, images):
        return NodeW(name).images([(names, size * MB) for names, size in images])

    n403002000 = [(["gcr.io/40:latest", "gcr.io/40:v1", "gcr.io/40:v1"], 40),
                  (["gcr.io/300:latest", "gcr.io/300:v1"], 300), (["gcr.io/2000:latest"], 2000)]
    n25010 = [(["gcr.io/250:latest"], 250), (["gcr.io/10:latest", "gcr.io/10:v1"], 10)]
    n60040900 = [(["gcr.io/600:latest"], 600), (["gcr.io/40:latest"], 40), (["gcr.io/900:latest"], 900)]
    n300600900 = [(["gcr.io/300:latest"], 300), (["gcr.io/600:latest"], 600), (["gcr.io/900:latest"], 900)]
    n400030 = [(["gcr.io/4000:latest"], 4000), (["gcr.io/30:latest"], 30)]
    n203040 = [(["gcr.io/20:latest"], 20), (["gcr.io/30:latest"], 30), (["gcr.io/40:latest"], 40)]

    def p(images, init=(), vols=()):
        w = pod()
        for im in images:
            w.container(image=im)
        for im in init:
            w.o["spec"].setdefault("initContainers", []).append({"name": "i", "image": im})
        for v in vols:
            w.image_volume(v)
        return w

    C = []
    C.append(score_case(src + ":255", "two images spread on two nodes, prefer the larger image one",
                        [node("node1", n403002000), node("node2", n25010)], p(["gcr.io/40", "gcr.io/250"]), IL,
                        [0, 5], norm=False))
    C.append(score_case(src + ":268", "two images on one node, prefer this node",
                        [node("node1", n403002000), node("node2", n25010)], p(["gcr.io/40", "gcr.io/300"]), IL,
                        [7, 0], norm=False))
    C.append(score_case(src + ":280", "if exceed limit, use limit",
                        [node("node1", n400030), node("node2", n25010)], p(["gcr.io/10", "gcr.io/4000"]), IL,
                        [100, 0], norm=False))
    C.append(score_case(src + ":295", "if exceed limit, use limit (with node which has no images present)",
                        [node("node1", n400030), node("node2", n25010), node("node3", [])],
                        p(["gcr.io/10", "gcr.io/4000"]), IL, [66, 0, 0], norm=False))
    C.append(score_case(src + ":310", "pod with multiple large images, node2 is preferred",
                        [node("node1", n60040900), node("node2", n300600900), node("node3", [])],
                        p(["gcr.io/300", "gcr.io/600", "gcr.io/900"]), IL, [32, 36, 0], norm=False))
    C.append(score_case(src + ":323", "pod with multiple small images",
                        [node("node1", n203040), node("node2", n400030)], p(["gcr.io/30", "gcr.io/40"]), IL,
                        [1, 0], norm=False))
    C.append(score_case(src + ":336", "pod with ImageVolume",
                        [node("node1", n300600900), node("node2", n400030)], p(["gcr.io/30"], vols=["gcr.io/300"]),
                        IL, [6, 0], norm=False))
    C.append(score_case(src + ":349", "same images as ImageVolume pod but as regular container images",
                        [node("node1", n300600900), node("node2", n400030)], p(["gcr.io/30", "gcr.io/300"]), IL,
                        [6, 0], norm=False))
    C.append(score_case(src + ":362", "include InitContainers",
                        [node("node1", n403002000), node("node2", n203040)], p(["gcr.io/30"], init=["gcr.io/300"]),
                        IL, [6, 0], norm=False))
    return C


# ---------------------------------------------------------------------------------------
# nodeports/node_ports_test.go:52-181
# ---------------------------------------------------------------------------------------
def node_ports_cases():
    src = "pkg/scheduler/framework/plugins/nodeports/node_ports_test.go"
    NP = "NodePorts"

    def newpod(*infos, uid=None):
        w = pod()
        ports = []
        for info in infos:
            proto, ip, port = info.split("/")
            ports.append({"hostIP": ip, "hostPort": int(port), "protocol": proto})
        w.container(ports=ports)
        return w

    def case(name, p, existing_infos, code=0, prefilter=0):
        n = NodeW("m1").capacity({"cpu": "4", "memory": "1Gi", "pods": "10"})
        ex = newpod(*existing_infos).node("m1") if existing_infos else None
        C.append(filter_case(src + ":52", name, [n], p, NP, [code], existing=[ex] if ex else [], prefilter=prefilter,
                             reasons=None if prefilter else [32 if code else 0]))

    C = []
    case("skip filter", pod(), [], prefilter=SKIP)
    case("other port", newpod("UDP/127.0.0.1/8080"), ["UDP/127.0.0.1/9090"])
    case("same udp port", newpod("UDP/127.0.0.1/8080"), ["UDP/127.0.0.1/8080"], code=U)
    case("same tcp port", newpod("TCP/127.0.0.1/8080"), ["TCP/127.0.0.1/8080"], code=U)
    case("different host ip", newpod("TCP/127.0.0.1/8080"), ["TCP/127.0.0.2/8080"])
    case("different protocol", newpod("UDP/127.0.0.1/8080"), ["TCP/127.0.0.1/8080"])
    case("second udp port conflict", newpod("UDP/127.0.0.1/8000", "UDP/127.0.0.1/8080"), ["UDP/127.0.0.1/8080"], code=U)
    case("first tcp port conflict", newpod("TCP/127.0.0.1/8001", "UDP/127.0.0.1/8080"),
         ["TCP/127.0.0.1/8001", "UDP/127.0.0.1/8081"], code=U)
    case("first tcp port conflict due to 0.0.0.0 hostIP", newpod("TCP/0.0.0.0/8001"), ["TCP/127.0.0.1/8001"], code=U)
    case("TCP hostPort conflict due to 0.0.0.0 hostIP", newpod("TCP/10.0.10.10/8001", "TCP/0.0.0.0/8001"),
         ["TCP/127.0.0.1/8001"], code=U)
    case("second tcp port conflict to 0.0.0.0 hostIP", newpod("TCP/127.0.0.1/8001"), ["TCP/0.0.0.0/8001"], code=U)
    case("second different protocol", newpod("UDP/127.0.0.1/8001"), ["TCP/0.0.0.0/8001"])
    case("UDP hostPort conflict due to 0.0.0.0 hostIP", newpod("UDP/127.0.0.1/8001"),
         ["TCP/0.0.0.0/8001", "UDP/0.0.0.0/8001"], code=U)
    nsc = pod()
    nsc.o["spec"]["initContainers"] = [{"name": "i", "ports": [{"containerPort": 8001, "hostPort": 8001,
                                                               "protocol": "TCP"}]}]
    case("non-sidecar initContainer using hostPort", nsc, ["TCP/0.0.0.0/8001"], prefilter=SKIP)
    sc = pod()
    sc.o["spec"]["initContainers"] = [{"name": "i", "restartPolicy": "Always",
                                       "ports": [{"containerPort": 8001, "hostPort": 8001, "protocol": "TCP"}]}]
    case("TCP hostPort conflict from sidecar initContainer", sc, ["TCP/0.0.0.0/8001"], code=U)
    return C


GROUPS = {
    "normalize_score": normalize_cases,
    "least_allocated": least_allocated_cases,
    "balanced_allocation": balanced_cases,
    "taint_toleration": taint_cases,
    "node_affinity_filter": node_affinity_filter_cases,
    "image_locality": image_locality_cases,
    "node_ports": node_ports_cases,
}


def main():
    extra = {}
    try:
        import make_fixtures_b  # second batch (PTS, IPA, Fit filter, scheduling cycles)
        extra = make_fixtures_b.GROUPS
    except ImportError:
        pass
    groups = dict(GROUPS)
    groups.update(extra)
    import make_fixtures_e  # fifth batch (Fit filter/scores, NodeAffinity score, NodeUnschedulable, NodeName)
    groups.update(make_fixtures_e.GROUPS)
    for name, fn in groups.items():
        cases = fn()
        path = os.path.join(HERE, f"{name}.json")
        with open(path, "w") as f:
            json.dump({"generated_by": "tests/golden/make_fixtures.py", "cases": cases}, f, indent=1, sort_keys=True)
        print(f"{path}: {len(cases)} cases")


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    main()

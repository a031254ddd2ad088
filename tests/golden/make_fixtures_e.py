"""Fifth fixture batch: NodeResourcesFit (filter and the three scoring strategies), NodeAffinity
scoring, NodeUnschedulable and NodeName, extracted from the reference's own tests by
tests/golden/gotable.py (the Go test files are read as text; the output is data only):

  noderesources/fit_test.go:149 TestEnoughRequests, :767 TestNotEnoughRequests,
    :823 TestStorageRequests, :880 TestRestartableInitContainers, :975 TestFitScore
  noderesources/most_allocated_test.go:38 TestMostAllocatedScoringStrategy
  noderesources/requested_to_capacity_ratio_test.go:41 TestRequestedToCapacityRatioScoringStrategy,
    :224 TestResourceBinPackingSingleExtended, :359 TestResourceBinPackingMultipleExtended
  nodeaffinity/node_affinity_test.go:936 TestNodeAffinityPriority
  nodeunschedulable/node_unschedulable_test.go:32 TestNodeUnschedulable
  nodename/node_name_test.go:32 TestNodeName

The fit_test.go helpers that are not single-return functions (newResourcePod, newResourceInitPod,
newResourceOverheadPod, newPodLevelResourcesPod -- fit_test.go:95-145, and makeNode --
util_test.go:43-57) are restated below with the same object shapes.  Cases are skipped (and
counted) when they need something outside the parity contract: the DRAExtendedResource gate,
the PodLevelResources gate turned off for a pod that sets pod-level resources, DRA objects.
Run through make_fixtures.py (it imports GROUPS from here).
"""
import copy
import os

from gotable import PAUSE, load_table

REF = "/root/reference"
PLUG = os.path.join(REF, "pkg/scheduler/framework/plugins")
R_TOO_MANY, R_CPU, R_MEM, R_EPH, R_SCALAR = 1 << 6, 1 << 7, 1 << 8, 1 << 9, 1 << 10
R_UNSCHED, R_NODE_NAME = 1 << 0, 1 << 1
SKIPPED = {}
_uid = [0]


def _src(rel, test):
    path = os.path.join(PLUG, rel)
    for i, line in enumerate(open(path), 1):
        if line.startswith(f"func {test}("):
            return f"pkg/scheduler/framework/plugins/{rel}:{i}"
    return f"pkg/scheduler/framework/plugins/{rel}"


def _skip(test, why):
    SKIPPED.setdefault(test, []).append(why)


# ---- fit_test.go:95-145 / util_test.go:43-57 restated ----------------------------------
def new_resource_pod(*usage):
    cs = []
    for r in usage:
        r = r or {}
        rl = {"cpu": f"{r.get('milliCPU', 0)}m", "memory": str(r.get("memory", 0)),
              "pods": str(r.get("allowedPodNumber", 0)), "ephemeral-storage": str(r.get("ephemeralStorage", 0))}
        for k, v in (r.get("scalarResources") or {}).items():
            rl[k] = str(v)
        cs.append({"name": "", "resources": {"requests": rl}})
    return {"spec": {"containers": cs}}


def new_resource_init_pod(pod, *usage):
    pod.setdefault("spec", {})["initContainers"] = new_resource_pod(*usage)["spec"]["containers"]
    return pod


def new_resource_overhead_pod(pod, overhead):
    pod.setdefault("spec", {})["overhead"] = {k: str(v) for k, v in overhead.items()}
    return pod


def new_pod_level_resources_pod(pod, res):
    pod.setdefault("spec", {})["resources"] = res
    return pod


def make_node(name, milli_cpu, memory, ext):
    rl = {k: str(v) for k, v in (ext or {}).items()}
    rl["cpu"] = f"{milli_cpu}m"
    rl["memory"] = str(memory)
    return {"metadata": {"name": name}, "status": {"capacity": dict(rl), "allocatable": dict(rl)}}


HELPERS = {"newResourcePod": new_resource_pod, "newResourceInitPod": new_resource_init_pod,
           "newResourceOverheadPod": new_resource_overhead_pod, "newPodLevelResourcesPod": new_pod_level_resources_pod,
           "makeNode": make_node}
CONSTS = {"ErrReasonUnschedulable": "node(s) were unschedulable",
          "ErrReason": "node(s) didn't match the requested node name"}


def _pod(p, node=None):
    p = copy.deepcopy(p or {})
    p.setdefault("apiVersion", "v1")
    p.setdefault("kind", "Pod")
    md = p.setdefault("metadata", {})
    if not md.get("uid"):
        _uid[0] += 1
        md["uid"] = f"e-{_uid[0]}"
    md.setdefault("name", md["uid"])
    if not md.get("namespace"):
        md["namespace"] = "default"
    spec = p.setdefault("spec", {})
    spec.setdefault("containers", [])
    if node is not None:
        spec["nodeName"] = node
    return p


def _node(n, name=None):
    n = copy.deepcopy(n or {})
    n.setdefault("apiVersion", "v1")
    n.setdefault("kind", "Node")
    md = n.setdefault("metadata", {})
    if name is not None:
        md["name"] = name
    n.setdefault("spec", {})
    n.setdefault("status", {})
    return n


def _reasons(status):
    bits = 0
    for r in (status or {}).get("reasons", []):
        if r == "Too many pods":
            bits |= R_TOO_MANY
        elif r == "Insufficient cpu":
            bits |= R_CPU
        elif r == "Insufficient memory":
            bits |= R_MEM
        elif r == "Insufficient ephemeral-storage":
            bits |= R_EPH
        elif r.startswith("Insufficient "):
            bits |= R_SCALAR
        elif r == CONSTS["ErrReasonUnschedulable"]:
            bits |= R_UNSCHED
        elif r == CONSTS["ErrReason"]:
            bits |= R_NODE_NAME
        else:
            raise ValueError(r)
    return bits


def _res_list(alloc):
    return {k: str(v) for k, v in alloc.items()}


def _fit_args(args):
    cfg = {}
    if args.get("ignoredResources"):
        cfg["ignoredResources"] = list(args["ignoredResources"])
    if args.get("ignoredResourceGroups"):
        cfg["ignoredResourceGroups"] = list(args["ignoredResourceGroups"])
    return {"nodeResourcesFit": cfg} if cfg else {}


def _filter_case(src, name, plugin, node, existing, pod, status, config=None):
    code = (status or {}).get("code", 0)
    return {"src": src, "name": name, "kind": "filter", "plugin": plugin, "config": config or {},
            "namespaces": [], "nodes": [node], "existing": existing, "pod": pod,
            "expect": {"prefilter": 0, "codes": [code], "reasons": [_reasons(status)]}}


# ---- NodeResourcesFit Filter ------------------------------------------------------------
def fit_filter_cases():
    rel = "noderesources/fit_test.go"
    out = []
    # node allocatable per harness: makeAllocatableResources(milliCPU, memory, pods, extendedA, storage, hugePageA)
    def alloc(cpu, mem, pods, ext, eph, huge):
        return {"cpu": f"{cpu}m", "memory": str(mem), "pods": str(pods), "example.com/aaa": str(ext),
                "ephemeral-storage": str(eph), "hugepages-2Mi": str(huge)}
    for test, table, node_alloc in (("testEnoughRequests", "enoughPodsTests", alloc(10, 20, 32, 5, 20, 5)),
                                    ("testNotEnoughRequests", "notEnoughPodsTests", alloc(10, 20, 1, 0, 0, 0)),
                                    ("testStorageRequests", "storagePodsTests", alloc(10, 20, 32, 5, 20, 5))):
        cases, _ = load_table(os.path.join(PLUG, rel), test, table=table, helpers=HELPERS)
        src = _src(rel, "T" + test[1:])
        for c in cases:
            if c["_unsupported"]:
                _skip(test, f"{c.get('name')}: {c['_unsupported']}")
                continue
            if c.get("draExtendedResourceEnabled"):
                _skip(test, f"{c['name']}: DRAExtendedResource gate")
                continue
            pod = _pod(c["pod"])
            if not c.get("podLevelResourcesEnabled") and pod["spec"].get("resources"):
                _skip(test, f"{c['name']}: PodLevelResources gate off")
                continue
            node = _node({"status": {"capacity": node_alloc, "allocatable": node_alloc}}, "node")
            existing = [_pod(p, "node") for p in c["nodeInfo"]["_nodeinfo_pods"]]
            out.append(_filter_case(src, c["name"], "NodeResourcesFit", node, existing, pod, c.get("wantStatus"),
                                    _fit_args(c.get("args") or {})))
    # testRestartableInitContainers (fit_test.go:880-973): its pods come from local closures; restated
    src = _src(rel, "TestRestartableInitContainers")
    node_alloc = {"cpu": "2m", "memory": "0", "pods": "1", "example.com/aaa": "0", "ephemeral-storage": "0",
                  "hugepages-2Mi": "0"}

    def sidecar_pod(req, side):
        c = {"name": "regular"}
        if req is not None:
            c["resources"] = {"requests": req}
        s = {"name": "restartable-init", "restartPolicy": "Always"}
        if side is not None:
            s["resources"] = {"requests": side}
        return {"spec": {"containers": [c], "initContainers": [s]}}
    rows = [("allow pod without restartable init containers", {"spec": {"containers": [{"name": "regular"}]}}, None),
            ("allow pod with restartable init containers", sidecar_pod(None, None), None),
            ("allow pod if the total requested resources do not exceed the node's allocatable resources",
             sidecar_pod({"cpu": "1m"}, {"cpu": "1m"}), None),
            ("not allow pod if the total requested resources do exceed the node's allocatable resources",
             sidecar_pod({"cpu": "1m"}, {"cpu": "2m"}), {"code": 3, "reasons": ["Insufficient cpu"]})]
    for name, pod, st in rows:
        node = _node({"status": {"capacity": {}, "allocatable": node_alloc}}, "node")
        out.append(_filter_case(src, name, "NodeResourcesFit", node, [], _pod(pod), st))
    return out


# ---- NodeResourcesFit Score: TestFitScore, MostAllocated, RequestedToCapacityRatio ---------
def _strategy(typ, resources, shape=None):
    s = {"type": typ}
    if resources is not None:
        s["resources"] = [{"name": r["name"], "weight": r.get("weight", 0)} for r in resources]
    if shape is not None:
        s["requestedToCapacityRatio"] = {"shape": [{"utilization": p.get("utilization", 0), "score": p.get("score", 0)}
                                                   for p in shape]}
    return {"nodeResourcesFit": {"scoringStrategy": s}}


def _score_case(src, name, nodes, existing, pod, config, want, status=0):
    names = [n["metadata"]["name"] for n in nodes]
    e = {"status": status}
    if status == 0:
        by = {s["name"]: s["score"] for s in want}
        e["raw"] = [by[n] for n in names]
    return {"src": src, "name": name, "kind": "score", "plugin": "NodeResourcesFit", "config": config,
            "namespaces": [], "nodes": nodes, "existing": existing, "pod": pod, "expect": e}


def _bound(pods, nodes):
    names = {n["metadata"]["name"] for n in nodes}
    return [_pod(p) for p in pods or [] if (p.get("spec") or {}).get("nodeName") in names]


def fit_score_cases():
    out = []
    rel = "noderesources/fit_test.go"
    cases, _ = load_table(os.path.join(PLUG, rel), "testFitScore", helpers=HELPERS)
    src = _src(rel, "TestFitScore")
    for c in cases:
        if c["_unsupported"] or c.get("draObjects"):
            _skip("TestFitScore", f"{c.get('name')}: {c['_unsupported'] or 'DRA objects'}")
            continue
        if not c.get("runPreScore"):
            # Score without PreScore recomputes the pod's requests from the spec
            # (fit.go:737-750 getPreScoreState fallback): the same numbers, so the case is kept
            pass
        strat = (c.get("nodeResourcesFitArgs") or {}).get("scoringStrategy") or {}
        rtcr = strat.get("requestedToCapacityRatio") or {}
        cfg = _strategy(strat.get("type", "LeastAllocated"), strat.get("resources"), rtcr.get("shape"))
        nodes = [_node(n) for n in c["nodes"]]
        out.append(_score_case(src, c["name"], nodes, _bound(c.get("existingPods"), nodes), _pod(c["requestedPod"]),
                               cfg, c["expectedPriorities"]))
    rel = "noderesources/most_allocated_test.go"
    cases, _ = load_table(os.path.join(PLUG, rel), "TestMostAllocatedScoringStrategy", helpers=HELPERS)
    src = _src(rel, "TestMostAllocatedScoringStrategy")
    for c in cases:
        bad = c["_unsupported"]
        res = c.get("resources")
        if res is None or any(r.get("weight", 0) == 0 for r in res):
            # the internal config type reaches NewFit undefaulted here; through the v1 configuration
            # SetDefaults_NodeResourcesFitArgs fills empty resources and 0 weights (v1/defaults.go:238-246)
            _skip("TestMostAllocatedScoringStrategy", f"{c.get('name')}: unreachable through v1 defaulting")
            continue
        if bad and bad.startswith("wantErrs"):  # a config the validation rejects (validation_pluginargs.go)
            out.append({"src": src, "name": c["name"], "kind": "config_error",
                        "config": _strategy("MostAllocated", c.get("resources"))})
            continue
        if bad:
            _skip("TestMostAllocatedScoringStrategy", f"{c.get('name')}: {bad}")
            continue
        nodes = [_node(n) for n in c["nodes"]]
        out.append(_score_case(src, c["name"], nodes, _bound(c.get("existingPods"), nodes), _pod(c["requestedPod"]),
                               _strategy("MostAllocated", c.get("resources")), c["expectedScores"],
                               c.get("wantStatusCode") or 0))
    rel = "noderesources/requested_to_capacity_ratio_test.go"
    cases, _ = load_table(os.path.join(PLUG, rel), "TestRequestedToCapacityRatioScoringStrategy", helpers=HELPERS)
    src = _src(rel, "TestRequestedToCapacityRatioScoringStrategy")
    shape = [{"utilization": 0, "score": 10}, {"utilization": 100, "score": 0}]  # :42-45
    for c in cases:
        if c["_unsupported"]:
            _skip("TestRequestedToCapacityRatioScoringStrategy", f"{c.get('name')}: {c['_unsupported']}")
            continue
        nodes = [_node(n) for n in c["nodes"]]
        out.append(_score_case(src, c["name"], nodes, _bound(c.get("existingPods"), nodes), _pod(c["requestedPod"]),
                               _strategy("RequestedToCapacityRatio", c.get("resources"), shape), c["expectedScores"]))
    for test, res, shp in (
            ("TestResourceBinPackingSingleExtended", [{"name": "intel.com/foo", "weight": 1}],  # :317-326
             [{"utilization": 0, "score": 0}, {"utilization": 100, "score": 1}]),
            ("TestResourceBinPackingMultipleExtended", [{"name": "intel.com/foo", "weight": 3},  # :547-557
                                                        {"name": "intel.com/bar", "weight": 5}],
             [{"utilization": 0, "score": 0}, {"utilization": 100, "score": 1}])):
        cases, _ = load_table(os.path.join(PLUG, rel), test, helpers=HELPERS)
        src = _src(rel, test)
        for c in cases:
            if c["_unsupported"]:
                _skip(test, f"{c.get('name')}: {c['_unsupported']}")
                continue
            nodes = [_node(n) for n in c["nodes"]]
            out.append(_score_case(src, c["name"], nodes, _bound(c.get("pods"), nodes), _pod(c["pod"]),
                                   _strategy("RequestedToCapacityRatio", res, shp), c["expectedScores"]))
    return out


# ---- NodeAffinity Score (TestNodeAffinityPriority) ----------------------------------------
def node_affinity_score_cases():
    rel = "nodeaffinity/node_affinity_test.go"
    test = "TestNodeAffinityPriority"
    cases, _ = load_table(os.path.join(PLUG, rel), test, helpers=HELPERS)
    src = _src(rel, test)
    out = []
    for c in cases:
        if c["_unsupported"]:
            _skip(test, f"{c.get('name')}: {c['_unsupported']}")
            continue
        cfg = {}
        if c.get("args"):
            if c["args"].get("addedAffinity"):
                cfg = {"nodeAffinity": {"addedAffinity": c["args"]["addedAffinity"]}}
        nodes = [_node(n) for n in c["nodes"]]
        names = [n["metadata"]["name"] for n in nodes]
        pod = _pod(c["pod"])
        pre = (c.get("wantPreScoreStatus") or {}).get("code", 0) if c.get("runPreScore") else 0
        na = ((pod["spec"].get("affinity") or {}).get("nodeAffinity") or {})
        added_pref = ((c.get("args") or {}).get("addedAffinity") or {}).get("preferredDuringSchedulingIgnoredDuringExecution")
        if not c.get("runPreScore") and not na.get("preferredDuringSchedulingIgnoredDuringExecution") and not added_pref:
            # the test scores without PreScore, which would Skip here (node_affinity.go:247-250); the
            # plugin contract at the boundary always runs PreScore first
            _skip(test, f"{c.get('name')}: Score without the PreScore that Skips")
            continue
        if pre:
            e = {"status": pre}  # PreScore Skip / Error (node_affinity.go:242-262)
        else:
            by = {s["name"]: s["score"] for s in c["expectedList"]}
            e = {"status": 0, "normalized": [by[n] for n in names]}
        disabled = not c.get("runPreScore")
        out.append({"src": src, "name": c["name"], "kind": "score", "plugin": "NodeAffinity", "config": cfg,
                    "namespaces": [], "nodes": nodes, "existing": [], "pod": pod, "expect": e,
                    **({"note": "runPreScore false: Score recomputes the preferred terms (node_affinity.go:270-276)"}
                       if disabled else {})})
    return out


# ---- NodeUnschedulable / NodeName Filter ---------------------------------------------------
def node_unschedulable_cases():
    rel = "nodeunschedulable/node_unschedulable_test.go"
    test = "TestNodeUnschedulable"
    cases, _ = load_table(os.path.join(PLUG, rel), test, table="testCases", extra_consts=CONSTS, helpers=HELPERS)
    src = _src(rel, test)
    out = []
    for c in cases:
        if c["_unsupported"]:
            _skip(test, f"{c.get('name')}: {c['_unsupported']}")
            continue
        out.append(_filter_case(src, c["name"], "NodeUnschedulable", _node(c["node"], "node"), [], _pod(c["pod"]),
                                c.get("wantStatus")))
    return out


def node_name_cases():
    rel = "nodename/node_name_test.go"
    test = "TestNodeName"
    cases, _ = load_table(os.path.join(PLUG, rel), test, extra_consts=CONSTS, helpers=HELPERS)
    src = _src(rel, test)
    out = []
    for c in cases:
        if c["_unsupported"]:
            _skip(test, f"{c.get('name')}: {c['_unsupported']}")
            continue
        node = _node(c["node"])
        if not node["metadata"].get("name"):
            node["metadata"]["name"] = "node"
        out.append(_filter_case(src, c["name"], "NodeName", node, [], _pod(c["pod"]), c.get("wantStatus")))
    return out


GROUPS = {
    "fit_filter": fit_filter_cases,
    "fit_score": fit_score_cases,
    "node_affinity_score": node_affinity_score_cases,
    "node_unschedulable": node_unschedulable_cases,
    "node_name": node_name_cases,
}

if __name__ == "__main__":
    for g, f in GROUPS.items():
        print(g, len(f()))
    for t, v in SKIPPED.items():
        print("skipped", t, len(v))
        for w in v:
            print("   ", w)

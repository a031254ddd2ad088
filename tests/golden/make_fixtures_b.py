"""Second fixture batch: PodTopologySpread and InterPodAffinity golden vectors, extracted from
the reference's own table-driven tests by tests/golden/gotable.py (which reads the Go test
files as text and evaluates their test tables into v1 JSON).  Output is data only.

Cases whose meaning depends on something the parity contract does not model are skipped
and counted: system-default spreading (Services/ReplicaSets in `objs`), feature gates the
case turns off while also setting the gated fields (NodeInclusionPolicy, MatchLabelKeys).
Run through make_fixtures.py (it imports GROUPS from here).
"""
import os

from gotable import load_table

REF = "/root/reference"
PLUG = os.path.join(REF, "pkg/scheduler/framework/plugins")
U, UU, SKIP, ERR = 2, 3, 5, 1

R_AFF, R_ANTI, R_EXIST = 1 << 13, 1 << 14, 1 << 15
R_PTS_LABEL, R_PTS_SKEW = 1 << 11, 1 << 12
REASONS = {"AFFINITY": R_AFF, "ANTI": R_ANTI, "EXISTING_ANTI": R_EXIST}
XCONST = {"ErrReasonExistingAntiAffinityRulesNotMatch": "EXISTING_ANTI",
          "ErrReasonAffinityRulesNotMatch": "AFFINITY", "ErrReasonAntiAffinityRulesNotMatch": "ANTI"}

_uid = [0]


def _rename_empty_ns(term):
    """The unit tests use the literal namespace "" (never defaulted there); both decoders
    default an empty namespace to "default", so "" is renamed consistently everywhere."""
    if isinstance(term, dict) and "namespaces" in term:
        term["namespaces"] = ["default" if n == "" else n for n in term["namespaces"]]


def _fix_pod(p, default_ns=None):
    import copy
    p = copy.deepcopy(p)
    md = dict(p.get("metadata") or {})
    if not md.get("uid"):
        _uid[0] += 1
        md["uid"] = f"gen-{_uid[0]}"
    if md.get("namespace", "") == "":
        md["namespace"] = "default"
    aff = (p.get("spec") or {}).get("affinity") or {}
    for kind in ("podAffinity", "podAntiAffinity"):
        for t in (aff.get(kind) or {}).get("requiredDuringSchedulingIgnoredDuringExecution") or []:
            _rename_empty_ns(t)
        for w in (aff.get(kind) or {}).get("preferredDuringSchedulingIgnoredDuringExecution") or []:
            _rename_empty_ns(w.get("podAffinityTerm"))
    p["metadata"] = md
    spec = dict(p.get("spec") or {})
    spec.setdefault("containers", [])
    p["spec"] = spec
    p.setdefault("apiVersion", "v1")
    p.setdefault("kind", "Pod")
    return p


def _bound(pods, nodes):
    """Existing pods, minus those bound to a node outside the case's node list: a scheduler
    snapshot only lists nodes that have a Node object (the unit tests' NewSnapshot keeps such
    ghost NodeInfos, which only work there because nothing ever matches their pods)."""
    names = {n["metadata"]["name"] for n in nodes}
    return [_fix_pod(p) for p in pods or [] if (p.get("spec") or {}).get("nodeName") in names]


def _fix_node(n):
    n = dict(n)
    n.setdefault("apiVersion", "v1")
    n.setdefault("kind", "Node")
    n.setdefault("spec", {})
    n.setdefault("status", {})
    return n


def _src(rel, test):
    path = os.path.join(PLUG, rel)
    for i, line in enumerate(open(path), 1):
        if line.startswith(f"func {test}("):
            return f"pkg/scheduler/framework/plugins/{rel}:{i}"
    return f"pkg/scheduler/framework/plugins/{rel}"


def _ns(name, labels=None):
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name, "labels": dict(labels or {})}}


def _has_policy(pod):
    return any("nodeAffinityPolicy" in c or "nodeTaintsPolicy" in c
               for c in (pod.get("spec") or {}).get("topologySpreadConstraints", []))


def _has_mlk(pod):
    return any(c.get("matchLabelKeys") for c in (pod.get("spec") or {}).get("topologySpreadConstraints", []))


# ---------------------------------------------------------------------------------------
# PodTopologySpread Filter (filtering_test.go TestSingleConstraint / TestMultipleConstraints)
# ---------------------------------------------------------------------------------------
def pts_filter_cases():
    out = []
    for test in ("TestSingleConstraint", "TestMultipleConstraints"):
        rel = "podtopologyspread/filtering_test.go"
        cases, _ = load_table(os.path.join(PLUG, rel), test)
        src = _src(rel, test)
        for c in cases:
            if c["_unsupported"]:
                continue
            pod = c["pod"]
            if not c.get("enableNodeInclusionPolicy") and _has_policy(pod):
                continue  # gate off + explicit policies: not the default-gates contract
            nodes = [_fix_node(n) for n in c["nodes"]]
            want = c.get("wantStatusCode") or {}
            if not want:
                continue
            out.append({
                "src": src, "name": c["name"], "kind": "filter", "plugin": "PodTopologySpread", "config": {},
                "namespaces": [], "nodes": nodes,
                "existing": _bound(c.get("existingPods"), nodes),
                "pod": _fix_pod(pod), "expect": {"prefilter": 0,
                                                  "codes": [want[n["metadata"]["name"]] for n in nodes]}})
    return out


# ---------------------------------------------------------------------------------------
# PodTopologySpread Score (scoring_test.go TestPodTopologySpreadScore)
# ---------------------------------------------------------------------------------------
def pts_score_cases():
    rel = "podtopologyspread/scoring_test.go"
    test = "TestPodTopologySpreadScore"
    cases, _ = load_table(os.path.join(PLUG, rel), test)
    src = _src(rel, test)
    out = []
    for c in cases:
        if c["_unsupported"] or c.get("objs"):
            continue
        pod = c["pod"]
        if not (pod.get("spec") or {}).get("topologySpreadConstraints"):
            continue  # system-default constraints need Services/ReplicaSets
        if not c.get("enableNodeInclusionPolicy") and _has_policy(pod):
            continue
        if not c.get("enableMatchLabelKeys") and _has_mlk(pod):
            continue
        nodes = [_fix_node(n) for n in c.get("nodes") or []]
        failed = [_fix_node(n) for n in c.get("failedNodes") or []]
        want = {s["name"]: s["score"] for s in c["want"]}
        out.append({
            "src": src, "name": c["name"], "kind": "score", "plugin": "PodTopologySpread", "config": {},
            "namespaces": [], "nodes": nodes + failed, "scored": [n["metadata"]["name"] for n in nodes],
            "existing": _bound(c.get("existingPods"), nodes + failed),
            "pod": _fix_pod(pod),
            "expect": {"status": 0, "normalized": [want[n["metadata"]["name"]] for n in nodes]}})
    return out


# ---------------------------------------------------------------------------------------
# InterPodAffinity Filter (filtering_test.go TestRequiredAffinitySingleNode / MultipleNodes)
# ---------------------------------------------------------------------------------------
def _status(s):
    if s is None:
        return 0, 0
    code = s["code"]
    bits = 0
    for r in s.get("reasons", []):
        bits |= REASONS.get(r, 0)
    return code, bits


def ipa_filter_cases():
    rel = "interpodaffinity/filtering_test.go"
    out = []
    score_ns = [_ns("subteam1.team1", {"team": "team1"}), _ns("subteam2.team1", {"team": "team1"}),
                _ns("subteam1.team2", {"team": "team2"}), _ns("subteam2.team2", {"team": "team2"})]
    for test in ("TestRequiredAffinitySingleNode", "TestRequiredAffinityMultipleNodes"):
        cases, _ = load_table(os.path.join(PLUG, rel), test, extra_consts=XCONST)
        src = _src(rel, test)
        for c in cases:
            if c["_unsupported"]:
                continue
            if test.endswith("SingleNode"):
                nodes = [_fix_node(c["node"])]
                wants = [c.get("wantFilterStatus")]
                namespaces = score_ns
            else:
                nodes = [_fix_node(n) for n in c["nodes"]]
                wants = c.get("wantFilterStatuses") or [None] * len(nodes)
                namespaces = [_ns("NS1")]
            pre = c.get("wantPreFilterStatus")
            pre_code = pre["code"] if pre else 0
            codes, reasons = zip(*[_status(w) for w in wants]) if wants else ((), ())
            e = {"prefilter": pre_code}
            if pre_code == 0:
                e["codes"] = list(codes)
                e["reasons"] = list(reasons)
            out.append({
                "src": src, "name": c["name"], "kind": "filter", "plugin": "InterPodAffinity", "config": {},
                "namespaces": namespaces, "nodes": nodes,
                "existing": _bound(c.get("pods"), nodes),
                "pod": _fix_pod(c["pod"]), "expect": e})
    return out


# ---------------------------------------------------------------------------------------
# InterPodAffinity Score (scoring_test.go TestPreferredAffinity / ...SymmetricWeight)
# ---------------------------------------------------------------------------------------
def ipa_score_cases():
    rel = "interpodaffinity/scoring_test.go"
    out = []
    namespaces = [_ns("subteam1.team1", {"team": "team1"}), _ns("subteam2.team1", {"team": "team1"}),
                  _ns("subteam1.team2", {"team": "team2"}), _ns("subteam2.team2", {"team": "team2"})]
    for test in ("TestPreferredAffinity", "TestPreferredAffinityWithHardPodAffinitySymmetricWeight"):
        cases, _ = load_table(os.path.join(PLUG, rel), test, extra_consts=XCONST)
        src = _src(rel, test)
        for c in cases:
            if c["_unsupported"]:
                continue
            cfg = {"interPodAffinity": {}}
            if test == "TestPreferredAffinity":
                cfg["interPodAffinity"]["hardPodAffinityWeight"] = 1
                if c.get("ignorePreferredTermsOfExistingPods"):
                    cfg["interPodAffinity"]["ignorePreferredTermsOfExistingPods"] = True
            else:
                cfg["interPodAffinity"]["hardPodAffinityWeight"] = c.get("hardPodAffinityWeight", 0)
            nodes = [_fix_node(n) for n in c["nodes"]]
            ws = c.get("wantStatus")
            status = ws["code"] if ws else 0
            e = {"status": status}
            if status == 0:
                want = {s["name"]: s["score"] for s in c.get("expectedList") or []}
                e["normalized"] = [want.get(n["metadata"]["name"], 0) for n in nodes]
            out.append({
                "src": src, "name": c["name"], "kind": "score", "plugin": "InterPodAffinity", "config": cfg,
                "namespaces": namespaces, "nodes": nodes,
                "existing": _bound(c.get("pods"), nodes),
                "pod": _fix_pod(c["pod"]), "expect": e})
    return out


GROUPS = {
    "pts_filter": pts_filter_cases,
    "pts_score": pts_score_cases,
    "ipa_filter": ipa_filter_cases,
    "ipa_score": ipa_score_cases,
}

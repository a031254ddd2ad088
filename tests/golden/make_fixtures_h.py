"""Eighth fixture batch: PodTopologySpread default constraints (plugin.go:46-57,
common.go:59-75, helper/spread.go:37-95, scoring.go:61-115 with requireAllTopologies = false).

Extracted by tests/golden/gotable.py from the reference's own tables (the Go files are read as text):

  scoring_test.go  TestPodTopologySpreadScore    the cases with `objs` (a Service selecting the pod;
                                                 the test's plugin is SystemDefaulting)
  scoring_test.go  TestPreScoreSkip              PreScore returns Skip (no soft constraints; default
                                                 constraints whose ReplicaSet does not exist)
  scoring_test.go  TestPreScoreStateEmptyNodes   see below
  filtering_test.go TestPreFilterState           the cases with defaultConstraints (ListDefaulting):
                                                 PreFilter Skip vs. constraints built

TestPreScoreStateEmptyNodes and TestPreFilterState compare the plugin's cycle state, which is not
observable through the FilterPlugin / ScorePlugin contract.  What is observable is transcribed:
PreFilter / PreScore Skip versus Success, and for PreScore the raw and normalised scores that the
expected state implies.  These cases have no existing pods, so every count in the expected state
is 0 and Score (scoring.go:199-226) reduces to round(sum over the constraints whose key the node
carries of (maxSkew - 1)), 0 for an ignored node; NormalizeScore (:229-268) follows.  Those two
restatements (`_raw_from_state`, `_normalize`) are the only derived numbers in this file, and each
case says so in its name suffix " [derived from want state]".

Namespace "" (the unit tests never default it) is renamed "default" for pods and objects alike,
as the other batches do.  Output: tests/golden/pts_defaults.json (data only).
Run:  python tests/golden/make_fixtures_h.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gotable import load_table as _load_table  # noqa: E402
from make_fixtures_b import PLUG, _bound, _fix_node, _fix_pod, _src  # noqa: E402

SKIP = 5

# the state tables' helpers, restated for the observable parts: a converted selector stays the
# LabelSelector it came from, labels.Nothing() a marker, sets are lists, weights keep their size
HELPERS = {"mustConvertLabelSelectorAsSelector": lambda t, sel: sel, "labels.Nothing": lambda: {"_nothing": True},
           "sets.New": lambda *a: list(a), "newCriticalPaths": lambda: {},
           "topologyNormalizingWeight": lambda n: {"_size": n}}


def load_table(path, test):
    return _load_table(path, test, extra_consts={"t": None}, helpers=HELPERS)


def _fix_obj(o):
    o = json.loads(json.dumps(o))
    md = dict(o.get("metadata") or {})
    if md.get("namespace", "") == "":
        md["namespace"] = "default"
    if not md.get("name"):
        md["name"] = f"{o['kind'].lower()}-{_fix_obj.n}"
        _fix_obj.n += 1
    o["metadata"] = md
    return o


_fix_obj.n = 0


def _pts_config(cfg):
    """config.PodTopologySpreadArgs -> the library's "podTopologySpread" block."""
    cfg = cfg or {}
    out = {"defaultingType": cfg.get("defaultingType") or "System"}
    if cfg.get("defaultConstraints"):
        out["defaultConstraints"] = cfg["defaultConstraints"]
    return {"podTopologySpread": out}


def _normalize(raw, ignored):
    """NormalizeScore (scoring.go:229-268)."""
    vals = [r for r, ig in zip(raw, ignored) if not ig]
    mn = min(vals) if vals else 0
    mx = max(vals) if vals else 0
    out = []
    for r, ig in zip(raw, ignored):
        if ig:
            out.append(0)
        elif mx == 0:
            out.append(100)
        else:
            out.append(100 * (mx + mn - r) // mx)
    return out


def _raw_from_state(nodes, want):
    """Score with all-zero counts (scoring.go:199-226): sum of (maxSkew - 1) over the keys the node carries."""
    ignored = set(want.get("ignoredNodes") or [])
    raw, ign = [], []
    for n in nodes:
        name = n["metadata"]["name"]
        labels = n["metadata"].get("labels") or {}
        if name in ignored:
            raw.append(0)
            ign.append(True)
            continue
        raw.append(sum(c["maxSkew"] - 1 for c in want["constraints"] if c["topologyKey"] in labels))
        ign.append(False)
    return raw, ign


def score_cases():
    rel = "podtopologyspread/scoring_test.go"
    out = []
    # TestPodTopologySpreadScore: the cases with objs (the others are in pts_score.json)
    src = _src(rel, "TestPodTopologySpreadScore")
    cases, _ = load_table(os.path.join(PLUG, rel), "TestPodTopologySpreadScore")
    for c in cases:
        if c["_unsupported"] or not c.get("objs"):
            continue
        nodes = [_fix_node(n) for n in c.get("nodes") or []]
        failed = [_fix_node(n) for n in c.get("failedNodes") or []]
        want = {s["name"]: s["score"] for s in c["want"]}
        out.append({
            "src": src, "name": c["name"], "kind": "score", "plugin": "PodTopologySpread",
            "config": _pts_config({"defaultingType": "System"}), "namespaces": [],
            "objects": [_fix_obj(o) for o in c["objs"]],
            "nodes": nodes + failed, "scored": [n["metadata"]["name"] for n in nodes],
            "existing": _bound(c.get("existingPods"), nodes + failed), "pod": _fix_pod(c["pod"]),
            "expect": {"status": 0, "normalized": [want[n["metadata"]["name"]] for n in nodes]}})
    # TestPreScoreSkip
    src = _src(rel, "TestPreScoreSkip")
    cases, _ = load_table(os.path.join(PLUG, rel), "TestPreScoreSkip")
    for c in cases:
        if c["_unsupported"]:
            continue
        nodes = [_fix_node(n) for n in c.get("nodes") or []]
        out.append({
            "src": src, "name": c["name"], "kind": "score", "plugin": "PodTopologySpread",
            "config": _pts_config(c.get("config")), "namespaces": [],
            "objects": [_fix_obj(o) for o in c.get("objs") or []], "nodes": nodes, "existing": [],
            "pod": _fix_pod(c["pod"]), "expect": {"status": SKIP}})
    # TestPreScoreStateEmptyNodes: scores implied by the expected preScoreState
    src = _src(rel, "TestPreScoreStateEmptyNodes")
    cases, _ = load_table(os.path.join(PLUG, rel), "TestPreScoreStateEmptyNodes")
    for c in cases:
        if c["_unsupported"]:  # counts are all 0: the inclusion-policy gate cannot change the scores
            continue
        nodes = [_fix_node(n) for n in c.get("nodes") or []]
        want = c["want"]
        raw, ign = _raw_from_state(nodes, want)
        out.append({
            "src": src, "name": c["name"] + " [derived from want state]", "kind": "score",
            "plugin": "PodTopologySpread", "config": _pts_config(c.get("config")), "namespaces": [],
            "objects": [_fix_obj(o) for o in c.get("objs") or []], "nodes": nodes, "existing": [],
            "pod": _fix_pod(c["pod"]), "expect": {"status": 0, "normalized": _normalize(raw, ign)}})
    return out


def filter_cases():
    rel = "podtopologyspread/filtering_test.go"
    src = _src(rel, "TestPreFilterState")
    cases, _ = load_table(os.path.join(PLUG, rel), "TestPreFilterState")
    out = []
    for c in cases:
        if c["_unsupported"] or not c.get("defaultConstraints"):
            continue
        nodes = [_fix_node(n) for n in c.get("nodes") or []]
        pre = c.get("wantPrefilterStatus")
        code = pre["code"] if pre else 0
        e = {"prefilter": code}
        if code == 0:
            # a pod with no existing matching pods: every node with the keys passes (skew 0 + self <= maxSkew
            # in these cases), a node without one is UnschedulableAndUnresolvable -- none of the transcribed
            # cases has nodes, so the codes list is the empty node list
            if nodes:
                continue
            e["codes"] = []
        out.append({
            "src": src, "name": c["name"], "kind": "filter", "plugin": "PodTopologySpread",
            "config": {"podTopologySpread": {"defaultingType": "List",
                                             "defaultConstraints": c["defaultConstraints"]}},
            "namespaces": [], "objects": [_fix_obj(o) for o in c.get("objs") or []], "nodes": nodes,
            "existing": _bound(c.get("existingPods"), nodes), "pod": _fix_pod(c["pod"]), "expect": e})
    return out


def config_cases():
    """validation_pluginargs_test.go TestValidatePodTopologySpreadArgs: the args the plugin's New() rejects.
    The table's wantErrs (field.ErrorList literals) is only read for presence: a case with it is a
    config the library must refuse, one without it a config it must accept."""
    rel = "pkg/scheduler/apis/config/validation/validation_pluginargs_test.go"
    test = "TestValidatePodTopologySpreadArgs"
    cases, _ = _load_table(os.path.join("/root/reference", rel), test, table="cases")
    src = rel
    for i, line in enumerate(open(os.path.join("/root/reference", rel)), 1):
        if line.startswith(f"func {test}("):
            src = f"{rel}:{i}"
    out = []
    for k, c in enumerate(cases):
        bad = c["_unsupported"]
        if bad and not bad.startswith("wantErrs:"):
            continue
        cfg = {"podTopologySpread": c["args"]}
        out.append({"src": src, "name": f"validation case {k}: {json.dumps(c['args'], sort_keys=True)}",
                    "kind": "config_error" if bad else "config_ok", "config": cfg})
    return out


def main():
    cases = score_cases() + filter_cases() + config_cases()
    path = os.path.join(HERE, "pts_defaults.json")
    with open(path, "w") as f:
        json.dump({"generated_by": "tests/golden/make_fixtures_h.py", "cases": cases}, f, indent=1, sort_keys=True)
    print(f"{path}: {len(cases)} cases")


if __name__ == "__main__":
    main()

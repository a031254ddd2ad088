"""Twelfth fixture batch: evaluateNominatedNode (SURVEY §8(a) A6's own-nomination part:
pkg/scheduler/schedule_one.go:657-669,714-745 -- a pod's status.nominatedNodeName is tried alone before the full
pass, and the one-feasible-node path of schedulePod, :586-598, places it there).

Extracted by tests/golden/gotable.py from the reference's own tables (the Go file is read as text):

  pkg/scheduler/schedule_one_test.go  TestEvaluateNominatedNode                3 cases
  pkg/scheduler/schedule_one_test.go  TestPreferNominatedNodeFilterCallCounts  3 cases

Both run findNodesThatFitPod / evaluateNominatedNode directly; here each case is a scheduling cycle of the pod
(ksg.h's ScheduleResult), with the expectations restated from the table's fields:

* TestEvaluateNominatedNode: no filter plugin is registered, so every node passes.  wantNodeList [n] -> the cycle
  places the pod on n with EvaluatedNodes 1 (FeasibleNodes 1).  wantError (the name is in no snapshot) ->
  findNodesThatFitPod logs the error and runs the full pass: both nodes feasible.  The table's placement
  (PodGroup scheduling) has no counterpart here -- every snapshot node is in the placement -- so the case "present
  in the snapshot but not in the placement" places the pod on its nominated node (flagged "placement_adapted").
* TestPreferNominatedNodeFilterCallCounts: a fake filter (failing on the nodes of nodeReturnCodeMap) and an
  equal-score plugin over node1..node3.  Here NodeUnschedulable plays the fake filter (the failing node is
  spec.unschedulable) and ImageLocality the equal scorer (no images: 0 everywhere).  expectedCount filter calls
  -> EvaluatedNodes: 1 call = the nominated node alone passed (evaluated 1); 3 calls = the full pass (evaluated
  3); 4 calls = the nominated node failed alone, then the full pass (evaluated 3: NodeToStatus holds node1 once,
  feasible 2).
Output: tests/golden/nominated.json (kind "cycle", run by golden_runner on the oracle and the device).
Run:  python tests/golden/make_fixtures_l.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gotable import load_table  # noqa: E402

REF = "/root/reference"
SRC = "pkg/scheduler/schedule_one_test.go"
ALL = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
       "PodTopologySpread", "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"]


def _named(pod, name):
    pod = json.loads(json.dumps(pod))
    pod["metadata"].setdefault("name", name)
    pod["metadata"].setdefault("namespace", "default")
    pod["metadata"].setdefault("uid", name)
    return pod


def main():
    consts = {"highPriority": 1000, "lowPriority": 0, "fwk.Unschedulable": 2}
    cases = []
    rows, _ = load_table(os.path.join(REF, SRC), "TestEvaluateNominatedNode", extra_consts=consts)
    for k, r in enumerate(rows):
        assert r["_unsupported"] is None, r
        nnn = r["pod"]["status"]["nominatedNodeName"]
        names = [n["metadata"]["name"] for n in r["allNodes"]]
        case = {"src": f"{SRC} TestEvaluateNominatedNode", "name": f"TestEvaluateNominatedNode[{k}] nominated {nnn}",
                "kind": "cycle", "config": {"disabledPlugins": [p for p in ALL if p != "ImageLocality"]},
                "namespaces": [], "nodes": r["allNodes"], "existing": [], "pod": _named(r["pod"], f"p{k}")}
        if r.get("wantError"):
            case["expect"] = {"status": 0, "evaluated": len(names), "feasible": len(names), "node_in": names}
        else:
            want = r.get("wantNodeList") or [nnn]
            case["expect"] = {"status": 0, "node": want[0], "evaluated": 1, "feasible": 1}
            if nnn not in r["placementNodes"]:
                case["placement_adapted"] = True
        cases.append(case)
    rows, _ = load_table(os.path.join(REF, SRC), "TestPreferNominatedNodeFilterCallCounts", extra_consts=consts)
    for r in rows:
        assert r["_unsupported"] is None, r
        fail = set((r.get("nodeReturnCodeMap") or {}).keys())
        nodes = [{"apiVersion": "v1", "kind": "Node", "metadata": {"name": n}, "spec": {"unschedulable": True} if n in fail else {}}
                 for n in ("node1", "node2", "node3")]  # makeNodeList: bare nodes
        nominated = r["pod"].get("status", {}).get("nominatedNodeName", "")
        calls = r["expectedCount"]
        if nominated and nominated not in fail:
            assert calls == 1
            expect = {"status": 0, "node": nominated, "evaluated": 1, "feasible": 1}
        else:
            full = calls - (1 if nominated else 0)  # the nominated node's lone call, then one per node
            assert full == 3
            expect = {"status": 0, "evaluated": full, "feasible": full - len(fail),
                      "node_in": [n["metadata"]["name"] for n in nodes if n["metadata"]["name"] not in fail]}
        cases.append({"src": f"{SRC} TestPreferNominatedNodeFilterCallCounts", "name": r["name"], "kind": "cycle",
                      "config": {"disabledPlugins": [p for p in ALL if p not in ("NodeUnschedulable", "ImageLocality")]},
                      "namespaces": [], "nodes": nodes, "existing": [], "pod": _named(r["pod"], "p"),
                      "expect": expect, "filter_calls": calls})
    with open(os.path.join(HERE, "nominated.json"), "w") as f:
        json.dump({"source": SRC, "cases": cases}, f, indent=1)
    print(f"nominated.json: {len(cases)} cases")


if __name__ == "__main__":
    main()

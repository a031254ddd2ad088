"""Tenth fixture batch: OpportunisticBatching's state machine (SURVEY §8(f) rank 4:
pkg/scheduler/framework/runtime/batch.go:65-229 -- GetNodeHint, StoreScheduleResults, batchStateCompatible).

Extracted by tests/golden/gotable.py from the reference's own table (the Go file is read as text):

  pkg/scheduler/framework/runtime/batch_test.go  TestBatchBasic   all 11 cases

Each case keeps the table's fields: the two pods' ids (the test plugin rejects a node for a pod whose id
starts with 'b' when the node already holds such a pod, batch_test.go:119-131), signatures, chosen nodes, the
sorted-node lists handed to StoreScheduleResults (testSortedScoredNodes: pop from the front), the cycle
relation (skipPod: a pod of another profile came between; sameCycle: one PodGroup cycle), the second pod's
nominated node, the GenericWorkload gate, and the expected hint and batch state.  The oracle runs each case
through its OpportunisticBatch restatement (ksgo_debug_batch_basic).
Output: tests/golden/batch_basic.json (data only; not a ksg.h cycle, so golden_runner.load_cases skips it).
Run:  python tests/golden/make_fixtures_j.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gotable import load_table  # noqa: E402

REF = "/root/reference"
SRC = "pkg/scheduler/framework/runtime/batch_test.go"


def _nodes(v):
    return None if v is None else list(v["nodes"])


def main():
    rows, _ = load_table(os.path.join(REF, SRC), "TestBatchBasic",
                         extra_consts={"blockingPodPrefix": "b", "nonBlockingPodPrefix": "a"})
    cases = []
    for r in rows:
        assert r["_unsupported"] is None, r
        st = r.get("expectedState")
        cases.append({
            "name": r["name"], "src": f"{SRC} TestBatchBasic", "kind": "batch_basic",
            "firstPodID": r["firstPodID"], "firstSig": r["firstSig"],
            "firstPodScheduledSuccessfully": bool(r.get("firstPodScheduledSuccessfully")),
            "firstChosenNode": r.get("firstChosenNode", ""), "firstOtherNodes": _nodes(r.get("firstOtherNodes")),
            "sameCycle": bool(r.get("sameCycle")), "skipPod": bool(r.get("skipPod")),
            "secondPodID": r["secondPodID"], "secondPodNominatedNodeName": r.get("secondPodNominatedNodeName", ""),
            "secondSig": r["secondSig"], "secondChosenNode": r.get("secondChosenNode", ""),
            "secondOtherNodes": _nodes(r.get("secondOtherNodes")),
            "genericWorkloadEnabled": bool(r.get("genericWorkloadEnabled")),
            "expectedHint": r["expectedHint"],
            "expectedState": None if st is None else {"signature": st["signature"],
                                                      "sortedNodes": _nodes(st["sortedNodes"])},
        })
    with open(os.path.join(HERE, "batch_basic.json"), "w") as f:
        json.dump({"source": SRC, "cases": cases}, f, indent=1)
    print(f"batch_basic.json: {len(cases)} cases")


if __name__ == "__main__":
    main()

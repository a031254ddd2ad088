"""Third fixture batch: percentageOfNodesToScore (numFeasibleNodesToFind) and the rotation of
nextStartNodeIndex, transcribed as data from the reference's scheduler tests:

  TestNumFeasibleNodesToFind   pkg/scheduler/schedule_one_test.go:4371-4437
  TestFairEvaluationForNodes   pkg/scheduler/schedule_one_test.go:4439-4486

The reference tests call numFeasibleNodesToFind directly; here each row becomes a scheduling
cycle over numAllNodes identical, all-feasible nodes, so the feasible list length is exactly
numNodesToFind (and, with every node feasible, so is EvaluatedNodes = processedNodes).  The
profile/global split collapses to the one effective percentage (profile if set, else global,
schedule_one.go:867-872).  TestFairEvaluationForNodes' rotation check (nextStartNodeIndex after
pod i == (i+1)*nodesToFind % numAllNodes) is observed through the chosen node: every node scores
the same, so the heap root -- the first node of the rotated feasible list -- is the node at
nextStartNodeIndex when the cycle starts.  Output is data only (tests/golden/sampling.json).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/schedule_one_test.go"

# (name, globalPercentage, profilePercentage or None, numAllNodes, wantNumNodes)  :4379-4424
NUM_FEASIBLE = [
    ("not set percentageOfNodesToScore and nodes number not more than 50", 0, None, 10, 10),
    ("set profile percentageOfNodesToScore and nodes number not more than 50", 0, 40, 10, 10),
    ("not set percentageOfNodesToScore and nodes number more than 50", 0, None, 1000, 420),
    ("set profile percentageOfNodesToScore and nodes number more than 50", 0, 40, 1000, 400),
    ("set global and profile percentageOfNodesToScore and nodes number more than 50", 100, 40, 1000, 400),
    ("set global percentageOfNodesToScore and nodes number more than 50", 40, None, 1000, 400),
    ("not set profile percentageOfNodesToScore and nodes number more than 50*125", 0, None, 6000, 300),
    ("set profile percentageOfNodesToScore and nodes number more than 50*125", 0, 40, 6000, 2400),
]

ROW_LINES = [4380, 4385, 4391, 4396, 4402, 4409, 4415, 4420]  # each row's `name:` line

NODE = {"metadata": {"name": "{i}"},
        "status": {"allocatable": {"cpu": "4", "memory": "32Gi", "pods": "110"},
                   "capacity": {"cpu": "4", "memory": "32Gi", "pods": "110"}}}
POD = {"metadata": {"name": "p", "namespace": "default", "uid": "p"},
       "spec": {"containers": [{"name": "c", "image": "pause"}]}}


def cases():
    out = []
    for line, (name, glob, prof, n, want) in zip(ROW_LINES, NUM_FEASIBLE):
        pct = prof if prof is not None else glob
        out.append({"name": name, "src": f"{SRC}:{line}", "kind": "cycle",
                    "config": {"percentageOfNodesToScore": pct},
                    "nodes_gen": {"count": n, "template": NODE}, "nodes": [], "pod": POD,
                    "expect": {"status": 0, "feasible": want, "evaluated": want}})
    # TestFairEvaluationForNodes :4439-4486 -- 500 nodes, percentage 30, 2*(500/150+1) cycles
    num_all, pct = 500, 30
    to_find = max(100, num_all * pct // 100)
    steps = [{"node": str((i * to_find) % num_all), "feasible": to_find, "evaluated": to_find}
             for i in range(2 * (num_all // to_find + 1))]
    out.append({"name": "fair evaluation for nodes", "src": f"{SRC}:4439-4486", "kind": "sequence",
                "config": {"percentageOfNodesToScore": pct},
                "nodes_gen": {"count": num_all, "template": NODE}, "nodes": [], "pod": POD,
                "expect": {"steps": steps}})
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "sampling.json"), "w") as f:
        json.dump({"source": "make_fixtures_c.py", "cases": cases()}, f, indent=1)
        f.write("\n")

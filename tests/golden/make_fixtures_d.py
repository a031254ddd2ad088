"""Fourth fixture batch: snapshot node order -- nodeTree (zone round-robin) and UpdateSnapshot's
list-rebuild rule -- transcribed as data from the reference's cache tests:

  TestNodeTree_AddNode / _RemoveNode / _UpdateNode   pkg/scheduler/backend/cache/node_tree_test.go:159-360
  TestNodeTree_List                                  node_tree_test.go:362-404
  TestNodeTreeMultiOperations                        node_tree_test.go:416-496
  TestSchedulerCache_UpdateSnapshot                  pkg/scheduler/backend/cache/cache_test.go:1814-2402
  TestSchedulerCache_updateNodeInfoSnapshotList      cache_test.go:2467-2613

Each case is a stream of cache events ("events" kind, tests/golden_runner.py) applied to a fresh
scheduler cache through the C ABI, with "snapshot" steps (UpdateSnapshot: ksg_num_nodes) and
the expected snapshot list after each.  How each expectation is read off the Go test:

* TestNodeTree_List / MultiOperations / updateNodeInfoSnapshotList assert the list verbatim.
* TestNodeTree_Add/Remove/UpdateNode assert the tree (zone -> nodes); every op runs before the
  first snapshot, so the snapshot list is nodeTree.list over that tree: zones in first-insertion
  order (a zone emptied by a removal leaves the order), round-robin across them.
* TestSchedulerCache_UpdateSnapshot asserts, after its final UpdateSnapshot, that the snapshot
  list equals nodeTree.list() (compareCacheWithNodeInfoSnapshot, cache_test.go:2418-2449).  Its
  nodes carry no zone labels, so that list is the AddNode order of the nodes still present.
  updatePod(i) is RemovePod + AddPod of the same pod (cache.go:469-474: priority changes only).
  Cases that only exercise PVCs, pod groups or snapshot-level assume (not modelled by the
  contract) are left out.

Plus cases derived from the list rule itself (cache.go:223-290; the reference's tests never move a
node between zones across a snapshot), marked "derived": a zone-changing UpdateNode keeps the
node's list position until a node is added or removed, and a node removed and re-added between
two snapshots keeps its position.  Output: tests/golden/snapshot_order.json (data only).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
TREE = "pkg/scheduler/backend/cache/node_tree_test.go"
CACHE = "pkg/scheduler/backend/cache/cache_test.go"
R, Z = "topology.kubernetes.io/region", "topology.kubernetes.io/zone"
BR, BZ = "failure-domain.beta.kubernetes.io/region", "failure-domain.beta.kubernetes.io/zone"
ALLOC = {"cpu": "1000m", "memory": "100m"}


def node(name, labels=None, alloc=None):
    return {"metadata": {"name": name, "labels": dict(labels or {})},
            "status": {"allocatable": dict(alloc or ALLOC)}}


# node_tree_test.go:29-136 allNodes
ALL = [
    node("node-0"),
    node("node-1", {R: "region-1"}),
    node("node-2", {Z: "zone-2"}),
    node("node-3", {R: "region-1", Z: "zone-2"}),
    node("node-4", {R: "region-1", Z: "zone-2"}),
    node("node-5", {R: "region-1", Z: "zone-3"}),
    node("node-6", {R: "region-2", Z: "zone-2"}),
    node("node-7", {R: "region-2", Z: "zone-2"}),
    node("node-8", {R: "region-2", Z: "zone-2"}),
    node("node-9", {R: "region-2", Z: "zone-2", BR: "region-2", BZ: "zone-2"}),
    node("node-10", {BR: "region-2", BZ: "zone-3"}),
]


def tree_list(zones):
    """nodeTree.list over an asserted tree: [(zone, [names])] in zone insertion order."""
    out = []
    k = 0
    while any(k < len(v) for _, v in zones):
        out += [v[k] for _, v in zones if k < len(v)]
        k += 1
    return out


def case(src, name, ops, derived=False):
    return {"src": src, "name": name, "kind": "events", "derived": derived, "nodes": [], "ops": ops}


def add(n):
    return {"op": "add_node", "node": n}


def rm(name, error=False):
    d = {"op": "remove_node", "name": name}
    if error:
        d["error"] = True
    return d


def upd(n):
    return {"op": "update_node", "node": n}


def snap(names):
    return {"op": "snapshot", "want": names}


def node_tree_cases():
    out = []
    src = f"{TREE}:159-217"
    out.append(case(src, "AddNode: single node no labels", [add(ALL[0]), snap(["node-0"])]))
    out.append(case(src, "AddNode: same node specified twice", [add(ALL[0]), add(ALL[0]), snap(["node-0"])]))
    out.append(case(src, "AddNode: mix of nodes with and without proper labels",
                    [add(n) for n in ALL[:4]] + [snap(tree_list(
                        [("", ["node-0"]), ("r1", ["node-1"]), ("z2", ["node-2"]), ("r1z2", ["node-3"])]))]))
    out.append(case(src, "AddNode: some zones with multiple nodes",
                    [add(n) for n in ALL[:7]] + [snap(tree_list(
                        [("", ["node-0"]), ("r1", ["node-1"]), ("z2", ["node-2"]), ("r1z2", ["node-3", "node-4"]),
                         ("r1z3", ["node-5"]), ("r2z2", ["node-6"])]))]))
    out.append(case(src, "AddNode: nodes also using deprecated zone/region label",
                    [add(n) for n in ALL[9:]] + [snap(tree_list([("r2z2", ["node-9"]), ("r2z3", ["node-10"])]))]))
    src = f"{TREE}:219-278"
    out.append(case(src, "RemoveNode: a single node with no labels",
                    [add(n) for n in ALL[:7]] + [rm("node-0")] + [snap(tree_list(
                        [("r1", ["node-1"]), ("z2", ["node-2"]), ("r1z2", ["node-3", "node-4"]), ("r1z3", ["node-5"]),
                         ("r2z2", ["node-6"])]))]))
    out.append(case(src, "RemoveNode: a few nodes including one from a zone with multiple nodes",
                    [add(n) for n in ALL[:7]] + [rm(f"node-{i}") for i in (1, 2, 3)] + [snap(tree_list(
                        [("", ["node-0"]), ("r1z2", ["node-4"]), ("r1z3", ["node-5"]), ("r2z2", ["node-6"])]))]))
    out.append(case(src, "RemoveNode: all nodes",
                    [add(n) for n in ALL[:7]] + [rm(f"node-{i}") for i in range(7)] + [snap([])]))
    out.append(case(src, "RemoveNode: non-existing node",
                    [rm(f"node-{i}", error=True) for i in range(5)] + [snap([])]))
    src = f"{TREE}:280-360"
    moved = node("node-0", {R: "region-1", Z: "zone-2"})
    out.append(case(src, "UpdateNode: a node without label",
                    [add(n) for n in ALL[:7]] + [upd(moved)] + [snap(tree_list(
                        [("r1", ["node-1"]), ("z2", ["node-2"]), ("r1z2", ["node-3", "node-4", "node-0"]),
                         ("r1z3", ["node-5"]), ("r2z2", ["node-6"])]))]))
    out.append(case(src, "UpdateNode: the only existing node", [add(ALL[0]), upd(moved), snap(["node-0"])]))
    out.append(case(src, "UpdateNode: non-existing node",
                    [add(ALL[0]), upd(node("node-new", {R: "region-1", Z: "zone-2"})), snap(["node-0", "node-new"])]))
    src = f"{TREE}:362-404"
    out.append(case(src, "List: empty tree", [snap([])]))
    out.append(case(src, "List: one node", [add(ALL[0]), snap(["node-0"])]))
    out.append(case(src, "List: four nodes", [add(n) for n in ALL[:4]] + [snap(["node-0", "node-1", "node-2", "node-3"])]))
    out.append(case(src, "List: all nodes", [add(n) for n in ALL[:9]] + [snap(
        ["node-0", "node-1", "node-2", "node-3", "node-5", "node-6", "node-4", "node-7", "node-8"])]))
    src = f"{TREE}:416-496"

    def multi(name, to_add, to_rm, ops, want):
        seq, a, r = [], 0, 0
        for op in ops:
            if op == "add":
                seq.append(add(to_add[a]))
                a += 1
            else:
                seq.append(rm(to_rm[r]["metadata"]["name"]))
                r += 1
        return case(src, "MultiOperations: " + name, seq + [snap(want)])
    out.append(multi("add and remove all nodes", ALL[2:9], ALL[2:9], ["add"] * 3 + ["remove"] * 3, []))
    out.append(multi("add and remove some nodes", ALL[2:9], ALL[2:9], ["add"] * 3 + ["remove"], ["node-3", "node-4"]))
    out.append(multi("remove three nodes", ALL[2:9], ALL[2:9], ["add"] * 3 + ["remove"] * 3 + ["add"], ["node-5"]))
    out.append(multi("add more nodes to an exhausted zone", ALL[4:9] + [ALL[3]], [], ["add"] * 6,
                     ["node-4", "node-5", "node-6", "node-3", "node-7", "node-8"]))
    out.append(multi("remove zone and add new", ALL[3:5] + ALL[6:8], ALL[3:5],
                     ["add", "add", "remove", "add", "add", "remove"], ["node-6", "node-7"]))
    return out


def cache_update_snapshot_cases():
    """cache_test.go:1814-2347: zone-less nodes test-node0..9, pods test-pod0..19 on node i%10."""
    src = f"{CACHE}:1814-2402"
    nodes = [node(f"test-node{i}") for i in range(10)]
    updated = [node(f"test-node{i}", alloc={"cpu": "2000m", "memory": "500m"}) for i in range(10)]

    def pod(i, aff=False):
        nm = f"p-affinity-{i}" if aff else f"test-pod{i}"
        uid = f"puid-affinity-{i}" if aff else f"test-puid{i}"
        p = {"metadata": {"name": nm, "namespace": "test-ns", "uid": uid},
             "spec": {"nodeName": f"test-node{i % 10 if not aff else i}", "containers": [{"name": "c", "image": "pause"}]}}
        if aff:  # PodAffinityExists("foo", "", required)
            p["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}, "topologyKey": ""}]}}
        return p

    A = lambda i: add(nodes[i])  # noqa: E731
    RM = lambda i: rm(f"test-node{i}")  # noqa: E731
    U = lambda i: upd(updated[i])  # noqa: E731
    AP = lambda i, aff=False: {"op": "add_pod", "pod": pod(i, aff)}  # noqa: E731
    RP = lambda i, aff=False: {"op": "remove_pod", "uid": pod(i, aff)["metadata"]["uid"]}  # noqa: E731
    UP = lambda i: [RP(i), AP(i)]  # noqa: E731
    S = {"op": "snapshot"}
    cases = [
        ("Empty cache", [], []),
        ("Single node", [A(1)], [1]),
        ("Add node, remove it, add it again", [A(1), S, RM(1), A(1)], [1]),
        ("Add node and remove it in the same cycle, add it again", [A(1), S, A(2), RM(1)], [2]),
        ("Add a few nodes, and snapshot in the middle", [A(0), S, A(1), S, A(2), S, A(3)], [0, 1, 2, 3]),
        ("Add a few nodes, and snapshot in the end", [A(0), A(2), A(5), A(6)], [0, 2, 5, 6]),
        ("Update some nodes", [A(0), A(1), A(5), S, U(1)], [0, 1, 5]),
        ("Add a few nodes, and remove all of them", [A(0), A(2), A(5), A(6), S, RM(0), RM(2), RM(5), RM(6)], []),
        ("Add a few nodes, and remove some of them", [A(0), A(2), A(5), A(6), S, RM(0), RM(6)], [2, 5]),
        ("Add a few nodes, remove all of them, and add more",
         [A(2), A(5), A(6), S, RM(2), RM(5), RM(6), S, A(7), A(9)], [7, 9]),
        ("Update nodes in particular order", [A(8), U(2), U(8), S, A(1)], [8, 2, 1]),
        ("Add some nodes and some pods", [A(0), A(2), A(8), S, AP(8), AP(2)], [0, 2, 8]),
        ("Updating a pod moves its node to the head", [A(0), AP(0), A(2), A(4)] + UP(0), [0, 2, 4]),
        ("Add pod before its node", [A(0), AP(1)] + UP(1) + [A(1)], [0, 1]),
        ("Remove node before its pods",
         [A(0), A(1), AP(1), AP(11), S, RM(1), S] + UP(1) + UP(11) + [RP(1), RP(11)], [0]),
        ("Add Pods with affinity", [A(0), AP(0, True), S, A(1)], [0, 1]),
        ("Add multiple nodes with pods with affinity", [A(0), AP(0, True), S, A(1), AP(1, True), S], [0, 1]),
        ("Add then Remove pods with affinity", [A(0), A(1), AP(0, True), S, RP(0, True), S], [0, 1]),
    ]
    out = []
    for name, ops, want in cases:
        seq = [dict(o) if o is not S else {"op": "snapshot"} for o in ops]
        seq.append(snap([f"test-node{i}" for i in want]))
        out.append(case(src, "UpdateSnapshot: " + name, seq))
    return out


def snapshot_list_cases():
    """cache_test.go:2467-2613: region/zone 0 holds node-0,1; region/zone 1 holds node-2..7."""
    src = f"{CACHE}:2467-2613"
    nodes = []
    for zone, nb in enumerate((2, 6)):
        for _ in range(nb):
            nodes.append(node(f"node-{len(nodes)}", {R: f"region-{zone}", Z: f"zone-{zone}"}))
    A = lambda i: add(nodes[i])  # noqa: E731
    S = {"op": "snapshot"}
    cases = [
        ("Empty cache", [], []),
        ("Single node", [A(0)], ["node-0"]),
        ("Two nodes", [A(0), S, A(1)], ["node-0", "node-1"]),
        ("bug 91601, two nodes, update the snapshot and add two nodes in different zones",
         [A(2), A(3), S, A(4), A(0)], ["node-2", "node-0", "node-3", "node-4"]),
        ("bug 91601, 6 nodes, one in a different zone",
         [A(2), A(3), A(4), A(5), S, A(6), A(0)], ["node-2", "node-0", "node-3", "node-4", "node-5", "node-6"]),
        ("bug 91601, 7 nodes, two in a different zone",
         [A(2), S, A(3), A(4), S, A(5), A(6), A(0), A(1)],
         ["node-2", "node-0", "node-3", "node-1", "node-4", "node-5", "node-6"]),
        ("bug 91601, 7 nodes, two in a different zone, different zone order",
         [A(2), A(1), S, A(3), A(4), S, A(5), A(6), A(0)],
         ["node-2", "node-1", "node-3", "node-0", "node-4", "node-5", "node-6"]),
    ]
    return [case(src, "updateNodeInfoSnapshotList: " + name, [dict(o) for o in ops] + [snap(want)])
            for name, ops, want in cases]


def derived_cases():
    """The list rule of UpdateSnapshot (cache.go:223-290) where the reference's tests do not go."""
    src = "pkg/scheduler/backend/cache/cache.go:223-290"
    a1, b2, c1, d1 = (node("a", {Z: "z1"}), node("b", {Z: "z2"}), node("c", {Z: "z1"}), node("d", {Z: "z1"}))
    a2 = node("a", {Z: "z2"})
    out = [
        case(src, "zone move keeps the list position until a node is added",
             [add(a1), add(b2), add(c1), snap(["a", "b", "c"]), upd(a2), snap(["a", "b", "c"]),
              add(d1), snap(["c", "b", "d", "a"])], derived=True),
        case(src, "zone move keeps the list position until a node is removed",
             [add(a1), add(b2), add(c1), snap(["a", "b", "c"]), upd(a2), snap(["a", "b", "c"]),
              rm("b"), snap(["c", "a"])], derived=True),
        case(src, "remove and re-add between snapshots keeps the position (map size unchanged)",
             [add(a1), add(b2), snap(["a", "b"]), rm("a"), add(a2), snap(["a", "b"]), rm("b"), snap(["a"])],
             derived=True),
        case(src, "a ghost node (pod before its node) joins the list when its node arrives",
             [add(a1), {"op": "add_pod", "pod": {"metadata": {"name": "g", "namespace": "default", "uid": "g"},
                                                 "spec": {"nodeName": "b", "containers": []}}},
              snap(["a"]), add(b2), snap(["a", "b"]), {"op": "remove_pod", "uid": "g"}, snap(["a", "b"])],
             derived=True),
        case(src, "a removed node with pods is a ghost; re-adding it rebuilds the list",
             [add(a1), add(b2), {"op": "add_pod", "pod": {"metadata": {"name": "g", "namespace": "default", "uid": "g"},
                                                          "spec": {"nodeName": "a", "containers": []}}},
              snap(["a", "b"]), rm("a"), snap(["b"]), add(a2), snap(["b", "a"]), rm("a", error=False),
              {"op": "remove_pod", "uid": "g"}, snap(["b"]), rm("a", error=True)], derived=True),
    ]
    return out


def cases():
    return node_tree_cases() + cache_update_snapshot_cases() + snapshot_list_cases() + derived_cases()


if __name__ == "__main__":
    with open(os.path.join(HERE, "snapshot_order.json"), "w") as f:
        json.dump({"source": "make_fixtures_d.py", "cases": cases()}, f, indent=1)
        f.write("\n")

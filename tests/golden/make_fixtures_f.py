"""Sixth fixture batch: whole scheduling cycles from the reference's scheduler tests
(pkg/scheduler/schedule_one_test.go), transcribed by hand as data where the case uses only in-tree
plugins:

  TestSchedulerSchedulePod :2922   "test podtopologyspread plugin - 2 nodes with maxskew=1" (:3194)
                                   "test podtopologyspread plugin - 3 nodes with maxskew=2" (:3224)
  Test_prioritizeNodes     :3961   "the score from Image Locality plugin with image in all nodes" (:4202)
                                   "... with image in partial nodes" (:4257)

The profile of each case enables exactly the plugins the test registers (everything else is in
"disabledPlugins").  Where the test registers a fake score plugin that gives every node the same
score (EqualPrioritizerPlugin), the profile has no score plugin: both make every feasible node tie,
so the heap root is the first feasible node either way, and the test's wantNodes set is the check.

Not transcribable: every other TestSchedulerSchedulePod case, TestFindFitAllError (:3782) and
TestFindFitSomeError register fake filter/score plugins (TrueFilter, MatchFilter, NumericMap,
...) whose behaviour no in-tree plugin has.  The FitError diagnosis they check -- every node's
status, code and failing plugin -- is checked here on a case "derived" from findNodesThatFitPod's
Diagnosis rule (schedule_one.go:622-712, 771-854: each failing node keeps its first failing
plugin's status) with an in-tree plugin, NodeResourcesFit, failing every node.
Output: tests/golden/schedule_cycles.json (data only).
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/schedule_one_test.go"
ALL = ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts", "NodeResourcesFit",
       "PodTopologySpread", "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"]
MB = 1024 * 1024
DEFAULT_MEMORY_REQUEST = 200 * MB  # schedutil.DefaultMemoryRequest (util/pod_resources.go:28-31)


def only(*keep):
    return {"disabledPlugins": [p for p in ALL if p not in keep]}


def node(name, labels=None, alloc=None, images=None):
    n = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": dict(labels or {})},
         "spec": {}, "status": {}}
    if alloc is not None:
        n["status"]["capacity"] = dict(alloc)
        n["status"]["allocatable"] = dict(alloc)
    if images is not None:
        n["status"]["images"] = images
    return n


def pod(name, uid, labels=None, node_name=None, spec=None):
    p = {"apiVersion": "v1", "kind": "Pod",
         "metadata": {"name": name, "namespace": "default", "uid": uid, "labels": dict(labels or {})},
         "spec": dict(spec or {"containers": []})}
    if node_name:
        p["spec"]["nodeName"] = node_name
    return p


def make_node(name, milli_cpu, memory, images=()):  # schedule_one_test.go:4620-4638
    return node(name, alloc={"cpu": f"{milli_cpu}m", "memory": str(memory), "pods": "100"}, images=list(images))


def pts_cases():
    spread = {"maxSkew": 1, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "DoNotSchedule",
              "labelSelector": {"matchExpressions": [{"key": "foo", "operator": "Exists"}]}}
    hn = lambda n: node(n, {"kubernetes.io/hostname": n})  # noqa: E731
    incoming = pod("p", "p", {"foo": ""}, spec={"containers": [], "topologySpreadConstraints": [spread]})
    out = [{
        "src": f"{SRC}:3194-3221", "name": "test podtopologyspread plugin - 2 nodes with maxskew=1", "kind": "cycle",
        "config": only("PodTopologySpread"), "namespaces": [], "nodes": [hn("node1"), hn("node2")],
        "existing": [pod("pod1", "pod1", {"foo": ""}, "node1")], "pod": incoming,
        "expect": {"status": 0, "node_in": ["node2"]}}]
    spread2 = dict(spread, maxSkew=2)
    incoming2 = pod("p", "p", {"foo": ""}, spec={"containers": [], "topologySpreadConstraints": [spread2]})
    out.append({
        "src": f"{SRC}:3224-3255", "name": "test podtopologyspread plugin - 3 nodes with maxskew=2", "kind": "cycle",
        "config": only("PodTopologySpread"), "namespaces": [], "nodes": [hn("node1"), hn("node2"), hn("node3")],
        "existing": [pod("pod1a", "pod1a", {"foo": ""}, "node1"), pod("pod1b", "pod1b", {"foo": ""}, "node1"),
                     pod("pod2", "pod2", {"foo": ""}, "node2")],
        "pod": incoming2, "expect": {"status": 0, "node_in": ["node2", "node3"]}})
    return out


def image_cases():
    img1 = [{"names": ["gcr.io/40:latest", "gcr.io/40:v1"], "sizeBytes": 80 * MB},  # :3962-3977
            {"names": ["gcr.io/300:latest", "gcr.io/300:v1"], "sizeBytes": 300 * MB}]
    img2 = [{"names": ["gcr.io/300:latest"], "sizeBytes": 300 * MB},  # :3979-3992
            {"names": ["gcr.io/40:latest", "gcr.io/40:v1"], "sizeBytes": 80 * MB}]
    img3 = [{"names": ["gcr.io/600:latest"], "sizeBytes": 600 * MB},  # :3994-4013
            {"names": ["gcr.io/40:latest"], "sizeBytes": 80 * MB},
            {"names": ["gcr.io/900:latest"], "sizeBytes": 900 * MB}]
    nodes = [make_node("node1", 1000, DEFAULT_MEMORY_REQUEST * 10, img1),
             make_node("node2", 1000, DEFAULT_MEMORY_REQUEST * 10, img2),
             make_node("node3", 1000, DEFAULT_MEMORY_REQUEST * 10, img3)]
    out = []
    for line, name, image, want in ((4202, "the score from Image Locality plugin with image in all nodes", "gcr.io/40",
                                     {"node1": 5, "node2": 5, "node3": 5}),
                                    (4257, "the score from Image Locality plugin with image in partial nodes",
                                     "gcr.io/300", {"node1": 18, "node2": 18, "node3": 0})):
        p = pod("p", f"p{line}", spec={"containers": [{"name": "c", "image": image}]})
        out.append({"src": f"{SRC}:{line}", "name": name, "kind": "cycle", "config": only("ImageLocality"),
                    "namespaces": [], "nodes": nodes, "existing": [], "pod": p,
                    "expect": {"status": 0, "plugin_scores": {"ImageLocality": want}, "totals": want}})
    return out


def fit_error_case():
    nodes = [make_node(n, 1000, DEFAULT_MEMORY_REQUEST * 10) for n in ("3", "2", "1")]
    p = pod("big", "big", spec={"containers": [{"name": "c", "resources": {"requests": {"cpu": "500m"}}}]})
    used = [pod(f"u{n}", f"u{n}", node_name=n, spec={"containers": [{"name": "c", "resources": {"requests": {"cpu": "600m"}}}]})
            for n in ("3", "2", "1")]
    return [{"src": "pkg/scheduler/schedule_one.go:622-712,771-854", "derived": True,
             "name": "FitError: every node rejected by its first failing plugin (analog of TestFindFitAllError :3782)",
             "kind": "cycle", "config": {}, "namespaces": [], "nodes": nodes, "existing": used, "pod": p,
             "expect": {"status": 2, "feasible": 0, "evaluated": 3,
                        "node_status": {n: [2, "NodeResourcesFit", 1 << 7] for n in ("1", "2", "3")}}}]


def cases():
    return pts_cases() + image_cases() + fit_error_case()


if __name__ == "__main__":
    with open(os.path.join(HERE, "schedule_cycles.json"), "w") as f:
        json.dump({"source": "make_fixtures_f.py", "cases": cases()}, f, indent=1)
        f.write("\n")

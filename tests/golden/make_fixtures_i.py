"""Ninth fixture batch: a pod's requests with in-place resize status (SURVEY §8(a) A25 / A21:
framework/types.go:1035-1076 CalculateResource with UseStatusResources, component-helpers
resource/helpers.go:151-304 PodRequests / AggregateContainerRequests / determineEffectiveRequests).

Extracted by tests/golden/gotable.py from the reference's own tables (the Go files are read as text):

  pkg/scheduler/framework/types_test.go  TestCalculatePodResourcesWithResize   all 9 cases
  component-helpers/resource/helpers_test.go  TestPodResourceRequests          every case whose options are
                                              {} or {UseStatusResources: bool} (ExcludeOverhead skipped)
  component-helpers/resource/helpers_test.go  TestAggregateContainerRequestsAndLimits  the requests half

The pods are built as the tests build them: TestCalculatePodResourcesWithResize's preparePodInfo
(types_test.go:2368-2446: container "c1", init container "i1", sidecar "s1" with restartPolicy Always,
their statuses under the same names, pod-level requests and status.resources, the resize conditions)
and the v1.Pod literals of the two helpers tests (helpers_test.go:872-885, :2643-2646).

Each case is kind "pod_resources" with "view":
  "calc"      CalculateResource: Requested MilliCPU / Memory / EphemeralStorage and Non0CPU / Non0Mem
              (the accounting of a bound or assumed pod, status resources included);
  "status"    PodRequests with UseStatusResources (the Requested half of "calc"; the tests' expected list);
  "spec"      PodRequests without status resources (Fit's PreFilter request, fit.go:317-325).
Expected quantities are converted as Resource.Add does (types.go: cpu MilliValue, the rest Value).
Output: tests/golden/pod_resources.json (data only).   Run:  python tests/golden/make_fixtures_i.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gotable import load_table, quantity_value  # noqa: E402

REF = "/root/reference"
TYPES = os.path.join(REF, "pkg/scheduler/framework/types_test.go")
HELPERS = os.path.join(REF, "staging/src/k8s.io/component-helpers/resource/helpers_test.go")
CONSTS = {"v1.PodResizePending": "PodResizePending", "v1.PodResizeInProgress": "PodResizeInProgress",
          "v1.ConditionTrue": "True", "v1.PodReasonDeferred": "Deferred", "v1.PodReasonInfeasible": "Infeasible",
          "v1.PodRunning": "Running"}


def _src(path, test):
    return f"{os.path.relpath(path, REF)} {test}"


def _pod(name, spec, status):
    status = {k: v for k, v in status.items() if v}
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "pod-resize-test", "uid": name},
            "spec": spec, "status": status}


def _amounts(rl):
    """ResourceList -> {cpu: MilliValue, memory / ephemeral-storage: Value}; None if it names others."""
    out = {"cpu": 0, "memory": 0, "ephemeral-storage": 0}
    for k, v in (rl or {}).items():
        if k not in out:
            return None
        out[k] = quantity_value(v, milli=(k == "cpu"))
    return out


def resize_cases():
    tab, _ = load_table(TYPES, "TestCalculatePodResourcesWithResize", extra_consts=CONSTS)
    out = []
    for i, c in enumerate(tab):
        assert not c["_unsupported"], c
        spec, status = {"containers": [], "initContainers": []}, {"phase": "Running", "containerStatuses": [],
                                                                  "initContainerStatuses": [], "conditions": []}
        # preparePodInfo (types_test.go:2368-2446)
        if c.get("podLevelRequests") is not None:
            spec["resources"] = {"requests": c["podLevelRequests"]}
        if c.get("podLevelStatusResources") is not None:
            status["resources"] = {"requests": c["podLevelStatusResources"]}
        spec["containers"].append({"name": "c1", "resources": {"requests": c.get("requests") or {}}})
        status["containerStatuses"].append({"name": "c1", "resources": {"requests": c.get("statusResources") or {}}})
        if c.get("initRequests") is not None:
            spec["initContainers"].append({"name": "i1", "resources": {"requests": c["initRequests"]}})
        if c.get("initStatusResources") is not None:
            status["initContainerStatuses"].append({"name": "i1", "resources": {"requests": c["initStatusResources"]}})
        if c.get("sidecarRequests") is not None:
            spec["initContainers"].append({"name": "s1", "resources": {"requests": c["sidecarRequests"]},
                                           "restartPolicy": "Always"})
        if c.get("sidecarStatusResources") is not None:
            status["initContainerStatuses"].append({"name": "s1", "resources": {"requests": c["sidecarStatusResources"]}})
        status["conditions"] = list(c.get("resizeStatus") or [])
        spec = {k: v for k, v in spec.items() if v}
        e = c["expectedResource"]
        want = {"cpu": e["resource"].get("milliCPU", 0), "memory": e["resource"].get("memory", 0),
                "ephemeral-storage": e["resource"].get("ephemeralStorage", 0),
                "non0_cpu": e.get("non0CPU", 0), "non0_mem": e.get("non0Mem", 0)}
        out.append({"name": c["name"], "src": _src(TYPES, "TestCalculatePodResourcesWithResize"), "kind": "pod_resources",
                    "view": "calc", "pod": _pod(f"resize-{i}", spec, status), "want": want})
    return out


def helpers_cases():
    out = []
    tab, _ = load_table(HELPERS, "TestPodResourceRequests", table="testCases", extra_consts=CONSTS)
    for i, c in enumerate(tab):
        assert not c["_unsupported"], c
        opts = c.get("options") or {}
        if set(opts) - {"useStatusResources"}:
            continue  # ExcludeOverhead: not a scheduler option
        want = _amounts(c.get("expectedRequests"))
        if want is None:
            continue
        spec = {"containers": c.get("containers") or [], "initContainers": c.get("initContainers") or []}
        if c.get("overhead"):
            spec["overhead"] = c["overhead"]
        status = {"containerStatuses": c.get("containerStatus"), "initContainerStatuses": c.get("initContainerStatuses"),
                  "conditions": c.get("podResizeStatus")}
        out.append({"name": c["description"], "src": _src(HELPERS, "TestPodResourceRequests"), "kind": "pod_resources",
                    "view": "status" if opts.get("useStatusResources") else "spec",
                    "pod": _pod(f"requests-{i}", spec, status), "want": want})
    tab, _ = load_table(HELPERS, "TestAggregateContainerRequestsAndLimits", table="cases", extra_consts=CONSTS)
    for i, c in enumerate(tab):
        assert not c["_unsupported"], c
        opts = c.get("options") or {}
        want = _amounts(c.get("expectedRequests"))
        if want is None:
            continue
        spec = {"containers": c.get("containers") or [], "initContainers": c.get("initContainers") or []}
        status = {"containerStatuses": c.get("containerStatuses"), "initContainerStatuses": c.get("initContainerStatuses")}
        out.append({"name": c["name"], "src": _src(HELPERS, "TestAggregateContainerRequestsAndLimits"),
                    "kind": "pod_resources", "view": "status" if opts.get("useStatusResources") else "spec",
                    "pod": _pod(f"aggregate-{i}", spec, status), "want": want})
    return out


def main():
    cases = resize_cases() + helpers_cases()
    with open(os.path.join(HERE, "pod_resources.json"), "w") as f:
        json.dump({"cases": cases}, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"pod_resources.json: {len(cases)} cases")


if __name__ == "__main__":
    main()

"""Eleventh fixture batch: OpportunisticBatching's pod signatures (which pod fields enter
frameworkImpl.SignPod, pkg/scheduler/framework/runtime/framework.go:884-924, and when a plugin refuses).

Extracted by tests/golden/gotable.py from the reference's own tables (the Go files are read as text):

  pkg/scheduler/framework/plugins/noderesources/fit_test.go                 testFitSignPod                 5 cases
  pkg/scheduler/framework/plugins/noderesources/balanced_allocation_test.go testBalancedAllocationSignPod  5 cases
  pkg/scheduler/framework/plugins/imagelocality/image_locality_test.go      TestImageSignature             3 cases
  pkg/scheduler/framework/plugins/podtopologyspread/filtering_test.go       TestPodTopoSignatures          3 cases
  pkg/scheduler/framework/plugins/interpodaffinity/plugin_test.go           TestPodAffinitySignature       3 cases
  pkg/scheduler/schedule_one_test.go                                        TestSignatures                 10 cases

Each plugin case keeps its pod, the plugin's arguments and the expected outcome: the fragments (signer key and
value; Fit / BalancedAllocation state theirs as computePodResourceRequest of the same pod, kept as that marker),
or a refusal (no fragments; a non-success status where the table names one).  TestSignatures' cases run
constant-signature test plugins through the framework: their plugin fragment lists, statuses and the expected
json bytes are kept as data for the framework rules (fragments merged by key, a refusing plugin makes the
signature nil).
Output: tests/golden/signatures.json (data only; tests/test_signatures.py runs it).
Run:  python tests/golden/make_fixtures_k.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gotable import load_table  # noqa: E402

REF = "/root/reference"
PL = "pkg/scheduler/framework/plugins/"
SIGNERS = {  # staging/src/k8s.io/kube-scheduler/framework/signers.go:34-45
    "fwk.DynamicResourcesSignerName": "v1.Pod.Spec.DynamicResources",
    "fwk.ImageNamesSignerName": "v1.Pod.Spec.CanonicalImageNames()",
    "fwk.LabelsSignerName": "v1.Pod.Labels",
    "fwk.NodeNameSignerName": "v1.Pod.Spec.NodeName",
    "fwk.NodeAffinitySignerName": "v1.Pod.Spec.Affinity.NodeAffinity",
    "fwk.NodeSelectorSignerName": "v1.Pod.Spec.Affinity.NodeSelector",
    "fwk.HostPortsSignerName": "v1.Pod.Spec.HostPorts()",
    "fwk.ResourcesSignerName": "v1.Pod.Spec.ContainerRequestsAndOverheads()",
    "fwk.SchedulerNameSignerName": "v1.Pod.Spec.SchedulerName",
    "fwk.TolerationsSignerName": "v1.Pod.Spec.Tolerations",
    "fwk.VolumesSignerName": "v1.Pod.Spec.Volumes.NonSyntheticSources()",
    "fwk.FeaturesSignerName": "v1.Pod.Spec.RequiredFeatures()",
}
HELPERS = {"computePodResourceRequest": lambda pod, opts: {"computePodResourceRequest": True}}
# the table's plugin -> the profile that runs only it (plus the volume / DRA / feature plugins every profile of
# this library carries, whose fragments are equal for every pod of these tables)
ONLY = ["NodeResourcesFit", "NodeResourcesBalancedAllocation", "ImageLocality", "PodTopologySpread", "InterPodAffinity",
        "TaintToleration", "NodeAffinity", "NodePorts", "NodeName", "NodeUnschedulable"]
TABLES = [
    ("NodeResourcesFit", PL + "noderesources/fit_test.go", "testFitSignPod", "expectedFragments"),
    ("NodeResourcesBalancedAllocation", PL + "noderesources/balanced_allocation_test.go", "testBalancedAllocationSignPod",
     "expectedFragments"),
    ("ImageLocality", PL + "imagelocality/image_locality_test.go", "TestImageSignature", "expectedSignature"),
    ("PodTopologySpread", PL + "podtopologyspread/filtering_test.go", "TestPodTopoSignatures", "expectedSignature"),
    ("InterPodAffinity", PL + "interpodaffinity/plugin_test.go", "TestPodAffinitySignature", "expectedSignature"),
]


def _config(plugin, args):
    cfg = {"disabledPlugins": [p for p in ONLY if p != plugin]}
    if plugin == "PodTopologySpread":
        cfg["podTopologySpread"] = dict(args or {})
    elif plugin == "InterPodAffinity":
        cfg["interPodAffinity"] = dict(args or {})
    return cfg


def _fragments(v):
    if v is None:
        return None
    out = []
    for f in v:
        val = f.get("value")
        if isinstance(val, dict) and val.get("computePodResourceRequest"):
            val = "computePodResourceRequest(pod)"
        out.append({"key": f["key"], "value": val})
    return out


def main():
    cases = []
    for plugin, src, test, field in TABLES:
        rows, _ = load_table(os.path.join(REF, src), test, extra_consts=SIGNERS, helpers=HELPERS)
        for k, r in enumerate(rows):
            assert r["_unsupported"] is None, (test, r["_unsupported"])
            frags = _fragments(r.get(field))
            ok_flag = r.get("scheduleable", r.get("schedulable"))
            code = r.get("expectedStatusCode")
            if code is not None:
                signable = code == 0
            elif ok_flag is not None:  # ("no affinity, ignore setting set": success, no fragments contributed)
                signable = bool(ok_flag)
            else:
                signable = frags is not None
            case = {"name": r.get("name") or f"{test}[{k}]", "src": f"{src} {test}", "plugin": plugin,
                    "pod": r["pod"], "config": _config(plugin, r.get("config")), "signable": signable,
                    "fragments": frags if signable else None}
            if "disableDRAExtendedResource" in r:
                # the DRA extended-resource mapping needs a DeviceClass this library's inputs never carry: the
                # enabled case is the reference's, kept with applies=false
                case["applies"] = bool(r["disableDRAExtendedResource"])
            cases.append(case)
    rows, _ = load_table(os.path.join(REF, "pkg/scheduler/schedule_one_test.go"), "TestSignatures", table="table",
                         extra_consts=SIGNERS)
    framework = []
    for r in rows:
        assert r["_unsupported"] is None, r["_unsupported"]
        exp = r.get("expectedSignature")
        framework.append({"name": r["name"], "src": "pkg/scheduler/schedule_one_test.go TestSignatures",
                          "plugins": [{"name": p["name"], "type": p["pluginType"], "fragments": _fragments(p.get("signature")),
                                       "code": p["status"]["code"]} for p in (r.get("plugins") or [])],
                          "expected": None if exp is None else json.loads(exp)})
    with open(os.path.join(HERE, "signatures.json"), "w") as f:
        json.dump({"source": "SignPod tables (see make_fixtures_k.py)", "cases": cases, "framework": framework}, f,
                  indent=1)
    print(f"signatures.json: {len(cases)} plugin cases, {len(framework)} framework cases")


if __name__ == "__main__":
    main()

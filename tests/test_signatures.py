"""OpportunisticBatching's pod signatures (SignPod, framework/runtime/framework.go:884-924) pinned by the
reference's own signature tables (tests/golden/signatures.json, made by make_fixtures_k.py from testFitSignPod,
testBalancedAllocationSignPod, TestImageSignature, TestPodTopoSignatures, TestPodAffinitySignature and
TestSignatures).  A signature decides whether a pod may take the previous pod's node hint (batch.go:183-200), so
what must match the reference is which pods sign alike and which do not sign at all.  Both the oracle
(ksgo_debug_pod_signature) and the product's own compile path (ksg_debug_pod_signature, libksg.so, host code:
no device needed) run every case.

The texts are each implementation's own encoding (one `|key=value` per signer key); equality of texts stands for
equality of the reference's json.Marshal bytes of the fragment map.
"""
import ctypes as C
import json
import os

import pytest

from oracle_binding import load as load_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = json.load(open(os.path.join(ROOT, "tests", "golden", "signatures.json")))
CASES = [c for c in FIX["cases"] if c.get("applies", True)]


def _product():
    from test_abi_cpu import _ensure_built
    lib = C.CDLL(_ensure_built())
    f = lib.ksg_debug_pod_signature
    f.restype = C.c_int
    f.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
    return f


def _oracle():
    f = load_oracle().ksgo_debug_pod_signature
    f.restype = C.c_int
    f.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]
    return f


IMPLS = {"oracle": _oracle, "product": _product}


def sign(fn, config, pod):
    """-> the signature text, or None for a nil signature.  (The tables' &v1.Pod{Spec: ...} literals carry no
    metadata; both decoders take API objects, which always do: a name is added, which no signer reads.)"""
    if "metadata" not in pod:
        pod = dict(pod, metadata={"name": "p"})
    c = json.dumps(config).encode()
    p = json.dumps(pod).encode()
    buf = C.create_string_buffer(1 << 16)
    n = C.c_size_t()
    rc = fn(c, len(c), p, len(p), buf, len(buf), C.byref(n))
    assert rc in (0, 1), f"rc={rc}"
    return buf.value.decode() if rc == 1 else None


@pytest.fixture(params=sorted(IMPLS), scope="module")
def impl(request):
    return IMPLS[request.param]()


@pytest.mark.parametrize("k", range(len(CASES)), ids=[f"{c['plugin']}:{c['name']}" for c in CASES])
def test_signable_as_the_reference(impl, k):
    """Each table case signs (fragments) or refuses (nil) as the reference's plugin does."""
    c = CASES[k]
    got = sign(impl, c["config"], c["pod"])
    assert (got is not None) == c["signable"], got


def _ref_value(c):
    return json.dumps(c["fragments"], sort_keys=True)


@pytest.mark.parametrize("plugin", sorted({c["plugin"] for c in CASES}))
def test_equality_classes_follow_the_reference(impl, plugin):
    """Within one table (one plugin's profile), two signable pods sign alike exactly when the reference's
    fragments are equal.  Fit / BalancedAllocation state theirs as computePodResourceRequest of the pod: the
    table's pods request pairwise different resources (1000m/2000, none, 500m+1500m/1000+3000 summed, and
    1000m/2000 plus one extended resource), so every case is its own class there."""
    cs = [c for c in CASES if c["plugin"] == plugin and c["signable"]]
    sigs = [sign(impl, c["config"], c["pod"]) for c in cs]
    for i in range(len(cs)):
        for j in range(len(cs)):
            if "computePodResourceRequest(pod)" in _ref_value(cs[i]):
                want = json.dumps(cs[i]["pod"], sort_keys=True) == json.dumps(cs[j]["pod"], sort_keys=True)
            else:
                want = _ref_value(cs[i]) == _ref_value(cs[j])
            assert (sigs[i] == sigs[j]) == want, (cs[i]["name"], cs[j]["name"], sigs[i], sigs[j])


def test_literal_fragment_values(impl):
    """The values the tables spell out: ImageLocality's sorted canonical names (myimage -> myimage:latest, two
    containers' images sorted), InterPodAffinity's labels, and no labels fragment with
    ignorePreferredTermsOfExistingPods."""
    by = {(c["plugin"], c["name"]): c for c in CASES}
    for name in ("no images", "one image", "two images unsorted"):
        c = by[("ImageLocality", name)]
        vals = c["fragments"][0]["value"]
        assert "|img=[" + "".join(v + "," for v in vals) + "]|" in sign(impl, c["config"], c["pod"])
    c = by[("InterPodAffinity", "no affinity, default settings")]
    lbl = c["fragments"][0]["value"]
    assert "|lbl={" + "".join(f"{k}={v};" for k, v in sorted(lbl.items())) + "}" in sign(impl, c["config"], c["pod"])
    c = by[("InterPodAffinity", "no affinity, ignore setting set")]
    assert "|lbl=" not in sign(impl, c["config"], c["pod"])
    # the two unsorted images sign as the sorted pair, and a repeated image once (a set: sets.List)
    pod = {"spec": {"containers": [{"name": "a", "image": "myimage"}, {"name": "b", "image": "zmyimage"},
                                   {"name": "c", "image": "myimage:latest"}]}}
    c = by[("ImageLocality", "two images unsorted")]
    assert sign(impl, c["config"], pod) == sign(impl, c["config"], c["pod"])


# ---- TestSignatures (schedule_one_test.go:1444): the framework's merge of the plugins' fragments -------------
FW = {c["name"]: c for c in FIX["framework"]}
ALL_OFF = ["NodeResourcesFit", "NodeResourcesBalancedAllocation", "ImageLocality", "PodTopologySpread",
           "InterPodAffinity", "TaintToleration", "NodeAffinity", "NodePorts", "NodeName", "NodeUnschedulable"]
POD = {"metadata": {"name": "foo", "labels": {"app": "x"}},
       "spec": {"schedulerName": "test-scheduler", "containers": [{"name": "c", "image": "img1",
                                                                     "resources": {"requests": {"cpu": "100m"}}}]}}


def _only(*keep):
    return {"disabledPlugins": [p for p in ALL_OFF if p not in keep],
            "podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}}


def test_framework_scheduler_name_alone(impl):
    """'no plugins': the scheduler name is the only pod-dependent fragment left (this library's profile always
    carries the volume / DRA / declared-feature plugins, whose fragments are equal for pods without volumes,
    claims or required features)."""
    assert FW["no plugins"]["expected"] == {"v1.Pod.Spec.SchedulerName": "test-scheduler"}
    a = sign(impl, _only(), POD)
    other = json.loads(json.dumps(POD))
    other["spec"]["containers"][0]["image"] = "img2"
    other["spec"]["containers"][0]["resources"]["requests"]["cpu"] = "900m"
    other["metadata"]["labels"] = {"app": "y"}
    assert a is not None and a == sign(impl, _only(), other)
    renamed = json.loads(json.dumps(POD))
    renamed["spec"]["schedulerName"] = "another"
    assert sign(impl, _only(), renamed) != a


def test_framework_fragments_of_two_plugins(impl):
    """'two plugins' / 'plugin with multiple fragments': every plugin's fragments enter the signature, so a pod
    differing in either plugin's input signs differently."""
    assert FW["two plugins"]["expected"] == {"test": 16, "test2": 17, "v1.Pod.Spec.SchedulerName": "test-scheduler"}
    cfg = _only("NodeResourcesFit", "ImageLocality")
    a = sign(impl, cfg, POD)
    img = json.loads(json.dumps(POD))
    img["spec"]["containers"][0]["image"] = "img2"
    req = json.loads(json.dumps(POD))
    req["spec"]["containers"][0]["resources"]["requests"]["cpu"] = "900m"
    assert len({a, sign(impl, cfg, img), sign(impl, cfg, req)}) == 3


def test_framework_overlapping_fragments(impl):
    """'overlapping fragments': two plugins giving the same key and value leave one fragment -- Fit and
    BalancedAllocation both sign ResourcesSignerName with computePodResourceRequest (fit.go:174-195,
    balanced_allocation.go:121-142), TaintToleration and NodeUnschedulable both TolerationsSignerName."""
    assert FW["overlapping fragments"]["expected"] == {"test": 16, "v1.Pod.Spec.SchedulerName": "test-scheduler"}
    assert sign(impl, _only("NodeResourcesFit"), POD) == sign(impl, _only("NodeResourcesBalancedAllocation"), POD) \
        == sign(impl, _only("NodeResourcesFit", "NodeResourcesBalancedAllocation"), POD)
    assert sign(impl, _only("TaintToleration"), POD) == sign(impl, _only("NodeUnschedulable"), POD) \
        == sign(impl, _only("TaintToleration", "NodeUnschedulable"), POD)


def test_framework_one_refusal_makes_nil(impl):
    """'unsignable plugin' / 'error plugin': one plugin's refusal makes the whole signature nil, whatever the
    others sign -- InterPodAffinity for a pod with affinity terms, PodTopologySpread for a pod with
    constraints, under the full default profile."""
    assert FW["unsignable plugin"]["expected"] is None and FW["error plugin"]["expected"] is None
    full = {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}}
    assert sign(impl, full, POD) is not None
    aff = json.loads(json.dumps(POD))
    aff["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"labelSelector": {"matchLabels": {"app": "x"}}, "topologyKey": "kubernetes.io/hostname"}]}}
    assert sign(impl, full, aff) is None
    tsc = json.loads(json.dumps(POD))
    tsc["spec"]["topologySpreadConstraints"] = [{"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule",
                                                 "labelSelector": {"matchLabels": {"app": "x"}}}]
    assert sign(impl, full, tsc) is None
    # System defaulting (the default): PodTopologySpread refuses every pod (podtopologyspread/plugin.go:92-102)
    assert sign(impl, {}, POD) is None


def test_product_and_oracle_agree_on_a_random_stream():
    """Beyond the tables: the product's and the oracle's signatures split a random pod stream into the same
    classes under the default plugins (List defaulting, so PodTopologySpread signs)."""
    from fuzz_gen import rand_cluster, rand_pod
    rng, cfg, nodes, existing, names = rand_cluster(911, n_nodes=20, n_existing=0)
    cfg = dict(cfg, podTopologySpread={"defaultingType": "List", "defaultConstraints": []})
    pods = [rand_pod(rng, k, names) for k in range(300)]
    o, p = _oracle(), _product()
    so = [sign(o, cfg, x) for x in pods]
    sp = [sign(p, cfg, x) for x in pods]
    assert [s is None for s in so] == [s is None for s in sp]
    co, cp = {}, {}
    assert [co.setdefault(s, len(co)) for s in so] == [cp.setdefault(s, len(cp)) for s in sp]
    assert sum(s is not None for s in so) > 10 and len(co) > 5

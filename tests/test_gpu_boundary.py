"""The boundary's former silent / context-killing limits, against the oracle (GPU).

* HostPortInfo has no size limit (kube-scheduler/framework/types.go:553-642): nodes holding more host
  ports than the mirror's initial row stride (8) must evaluate NodePorts exactly, and the context must
  keep working as ports come and go (the device row widens by a re-layout).
* Distinct extended resources beyond the initial 16 scalar columns are kept (NewResource,
  framework/types.go:1263-1291), not dropped.
* Pods whose volumes / resource claims need the volume plugins or DynamicResources are declined at
  ksg_pod_compile with KSG_ENOTSUP, and the context stays usable.
"""
import pytest

from ksg.abi import KSG_ENOTSUP, KsgError
from ksg.objects import NodeW, PodW
from oracle_binding import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from ksg.native import Scheduler
    return Scheduler


def _pair(native, nodes, existing=(), cfg=None):
    bs = []
    for make in (native, oracle):
        b = make(cfg or {})
        for n in nodes:
            b.add_node(n)
        for p in existing:
            b.add_pod(p)
        bs.append(b)
    assert bs[0].node_names() == bs[1].node_names()
    return bs


def _cycle(g, o, pod, tag):
    rg, eg = g.schedule_one(g.compile(pod), assume=True, evaluate=True)
    ro, eo = o.schedule_one(o.compile(pod), assume=True, evaluate=True)
    assert rg.as_tuple() == ro.as_tuple(), f"{tag}: {rg.as_tuple()} != {ro.as_tuple()}"
    assert eg == eo, f"{tag}: per-node evaluation differs"
    return rg


def _node(i, cap=None):
    return NodeW(f"n{i:03d}").capacity(cap or {"cpu": "64", "memory": "256Gi", "pods": "110"}) \
        .label("kubernetes.io/hostname", f"n{i:03d}").obj()


def test_node_with_many_host_ports(native):
    nodes = [_node(i) for i in range(40)]
    existing = []
    for k in range(12):  # twelve host ports on n000, three more on n001
        existing.append(PodW(f"e{k}", uid=f"e{k}").host_port(9000 + k).node("n000").obj())
    for k in range(3):
        existing.append(PodW(f"f{k}", uid=f"f{k}").host_port(9100 + k, proto="UDP").node("n001").obj())
    g, o = _pair(native, nodes, existing)
    for k in range(12):  # conflicting ports: n000 must be filtered out; free ports: anywhere
        p = PodW(f"p{k}", uid=f"p{k}").host_port(9000 + (k * 5) % 24).obj()
        _cycle(g, o, p, f"pod {k}")
    assert g.compare_mirror(sync=True)[0] == 0
    # ports leave and come back: the rows shrink / grow in place
    for k in range(0, 12, 2):
        g.remove_pod(f"e{k}")
        o.remove_pod(f"e{k}")
    for k in range(20):
        p = PodW(f"q{k}", uid=f"q{k}").host_port(9000 + k % 16).host_port(9300 + k).obj()
        _cycle(g, o, p, f"pod q{k}")
    assert g.compare_mirror(sync=True)[0] == 0


def test_batch_assumes_many_ports_onto_one_node(native):
    """A batch whose pods all carry distinct host ports and fit one node only: the device row must hold
    every port the batch's assumes add (the host widens it before the launch)."""
    nodes = [_node(0)] + [_node(i, {"cpu": "1", "memory": "1Gi", "pods": "110"}) for i in range(1, 6)]
    g, o = _pair(native, nodes)
    pods = [PodW(f"b{k}", uid=f"b{k}").container(requests={"cpu": "2"}).host_port(7000 + k).host_port(8000 + k).obj()
            for k in range(24)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"pod {k}"
    assert g.compare_mirror(sync=True)[0] == 0
    # every port is now taken on n000: a pod asking for one of them is rejected there
    _cycle(g, o, PodW("c", uid="c").container(requests={"cpu": "2"}).host_port(7005).obj(), "conflict")


def test_port_flush_and_dynamic_rows_stay_consistent(native):
    """a node over the initial port stride, its pod removed, then pods added to nodes flushed
    in the same batch of dynamic rows: the mirror must equal the cache."""
    nodes = [_node(i) for i in range(20)]
    g, o = _pair(native, nodes)
    for k in range(10):
        for b in (g, o):
            b.add_pod(PodW(f"h{k}", uid=f"h{k}").host_port(6000 + k).node("n003").obj())
    for b in (g, o):
        b.add_pod(PodW("x", uid="x").container(requests={"cpu": "1"}).node("n004").obj())
    _cycle(g, o, PodW("p0", uid="p0").host_port(6001).obj(), "after 10 ports")
    for b in (g, o):
        b.remove_pod("h3")
        b.add_pod(PodW("y", uid="y").container(requests={"cpu": "3"}).node("n004").obj())
        b.add_pod(PodW("z", uid="z").container(requests={"cpu": "5"}).node("n005").obj())
    assert g.compare_mirror(sync=True)[0] == 0
    for k in range(8):
        _cycle(g, o, PodW(f"r{k}", uid=f"r{k}").container(requests={"cpu": "7"}).host_port(6000 + k).obj(), f"r{k}")
    assert g.compare_mirror(sync=True)[0] == 0


def test_more_than_sixteen_extended_resources(native):
    res = [f"example.com/dev{k}" for k in range(22)]
    nodes = []
    for i in range(30):
        cap = {"cpu": "16", "memory": "64Gi", "pods": "110"}
        for k, r in enumerate(res):
            if (i + k) % 3:
                cap[r] = str((i * 7 + k) % 5)
        nodes.append(_node(i, cap))
    g, o = _pair(native, nodes)
    for k in range(30):
        r = res[16 + k % 6] if k % 2 else res[k % 16]
        p = PodW(f"p{k}", uid=f"p{k}").container(requests={"cpu": "500m", r: "1"}).obj()
        _cycle(g, o, p, f"pod {k} ({r})")
    assert g.compare_mirror(sync=True)[0] == 0
    # a node brought in later with a brand-new resource name
    late = dict({"cpu": "8", "memory": "8Gi", "pods": "110"}, **{"example.com/late": "2"})
    for b in (g, o):
        b.add_node(_node(99, late))
    _cycle(g, o, PodW("late", uid="late").container(requests={"example.com/late": "1"}).obj(), "late resource")


@pytest.mark.parametrize("volume", [
    {"name": "data", "persistentVolumeClaim": {"claimName": "c"}},
    {"name": "eph", "ephemeral": {"volumeClaimTemplate": {"spec": {}}}},
    {"name": "pd", "gcePersistentDisk": {"pdName": "d"}},
    {"name": "rbd", "rbd": {"monitors": ["m"], "image": "i"}},
])
def test_volume_pods_are_declined_and_context_stays_usable(native, volume):
    nodes = [_node(i) for i in range(10)]
    g, o = _pair(native, nodes)
    p = PodW("v", uid="v").container(requests={"cpu": "1"}).obj()
    p["spec"]["volumes"] = [{"name": "cfg", "configMap": {"name": "x"}}, volume]
    for b in (g, o):
        with pytest.raises(KsgError) as ex:
            b.compile(p)
        assert f"rc={KSG_ENOTSUP}" in str(ex.value)
    ok = PodW("ok", uid="ok").container(requests={"cpu": "1"}).obj()
    ok["spec"]["volumes"] = [{"name": "cfg", "configMap": {"name": "x"}}, {"name": "t", "emptyDir": {}}]
    for k in range(3):
        _cycle(g, o, dict(ok, metadata=dict(ok["metadata"], name=f"ok{k}", uid=f"ok{k}")), f"ok {k}")


def test_resource_claim_pods_are_declined(native):
    g, o = _pair(native, [_node(0)])
    p = PodW("d", uid="d").container(requests={"cpu": "1"}).obj()
    p["spec"]["resourceClaims"] = [{"name": "gpu", "resourceClaimName": "gpu-claim"}]
    for b in (g, o):
        with pytest.raises(KsgError):
            b.compile(p)
    _cycle(g, o, PodW("e", uid="e").container(requests={"cpu": "1"}).obj(), "after")


def test_generation_counts_cache_events(native):
    """ksg_generation (the plugin-level shim's check): every applied cache mutation -- node
    add / update / remove, bound pod add / remove, each assume of a scheduling call, a forget -- counts one
    event; rejected calls count none; the node-list generation moves when the snapshot list is rebuilt
    (a node added or removed), not for an in-place node update or pod events."""
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(300, 20, 40)
    s = native({})
    lg0, ev0 = s.generation()
    for n in nodes:
        s.add_node(n)
    for p in init:
        s.add_pod(p)
    lg1, ev1 = s.generation()
    assert ev1 - ev0 == len(nodes) + len(init)
    assert lg1 > lg0
    rs = s.schedule_batch([s.compile(p) for p in pods[:30]], assume=True)
    placed = sum(r.status == 0 for r in rs)
    h = s.compile(pods[30])
    r, _ = s.schedule_one(h, assume=True)
    placed += r.status == 0
    lg2, ev2 = s.generation()
    assert ev2 - ev1 == placed and lg2 == lg1
    s.forget(h)
    upd = dict(nodes[5])
    upd["metadata"] = dict(upd["metadata"], labels=dict(upd["metadata"].get("labels", {}), extra="x"))
    s.update_node(upd)
    s.remove_pod(init[0]["metadata"]["uid"])
    with pytest.raises(Exception):
        s.remove_pod("no-such-pod")
    lg3, ev3 = s.generation()
    assert ev3 - ev2 == 3 and lg3 == lg2
    s.remove_node(nodes[7]["metadata"]["name"])
    lg4, ev4 = s.generation()
    assert ev4 - ev3 == 1 and lg4 > lg3
    s.close()

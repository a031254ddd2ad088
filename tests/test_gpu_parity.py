"""Parity of the HIP path (libksg.so through the C ABI) against the CPU oracle.

Bar: bit-exact -- identical feasible sets, per-node Filter codes/plugins/reasons, per-plugin
weighted int64 score vectors, TotalScores, chosen node (incl. the heap tie-break), and
EvaluatedNodes/FeasibleNodes, over pod sequences where each assume lands before the next pod.
"""
import random

import pytest

from fuzz_gen import add_resize_status, namespaces, rand_cluster, rand_pod
from golden_runner import load_cases, run_case
from oracle_binding import oracle

pytestmark = pytest.mark.gpu

CASES = load_cases()


@pytest.fixture(scope="module")
def native():
    from ksg.native import Scheduler
    return Scheduler


@pytest.mark.parametrize("name,case", CASES, ids=[c[0] for c in CASES])
def test_golden_vectors_on_device(native, name, case):
    errs = run_case(native, case)
    assert not errs, f"{case['src']}: {errs}"


def _pair(native, cfg, nodes, existing):
    bs = []
    for make in (native, oracle):
        b = make(cfg)
        for ns in namespaces():
            b.upsert_namespace(ns)
        for n in nodes:
            b.add_node(n)
        for p in existing:
            b.add_pod(p)
        bs.append(b)
    assert bs[0].node_names() == bs[1].node_names()
    return bs


def _cmp_cycle(g, o, pod, tag, evaluate=True):
    hg, ho = g.compile(pod), o.compile(pod)
    rg, eg = g.schedule_one(hg, assume=True, evaluate=evaluate)
    ro, eo = o.schedule_one(ho, assume=True, evaluate=evaluate)
    assert rg.as_tuple() == ro.as_tuple(), f"{tag}: result {rg.as_tuple()} != oracle {ro.as_tuple()}"
    if evaluate:
        for k in eo:
            assert eg[k] == eo[k], f"{tag}: eval[{k}] differs"
    return hg, ho, rg


@pytest.mark.parametrize("seed", range(32))
def test_random_sequences_match_oracle(native, seed):
    rng, cfg, nodes, existing, names = rand_cluster(seed, n_nodes=rng_nodes(seed), n_existing=60)
    g, o = _pair(native, cfg, nodes, existing)
    for k in range(40):
        _cmp_cycle(g, o, rand_pod(rng, k, names), f"seed {seed} pod {k}")


def rng_nodes(seed):
    return [7, 60, 130, 257, 300, 600][seed % 6]


@pytest.mark.parametrize("seed", range(6))
def test_batch_matches_sequential_oracle(native, seed):
    rng, cfg, nodes, existing, names = rand_cluster(1000 + seed, n_nodes=513, n_existing=100)
    g, o = _pair(native, cfg, nodes, existing)
    pods = [rand_pod(rng, k, names) for k in range(150)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"seed {seed} pod {k}"


@pytest.mark.parametrize("seed", range(4))
def test_resized_bound_pods_match_oracle(native, seed):
    """Bound pods mid-resize (InPlacePodVerticalScaling, GA: container / pod-level status resources,
    allocatedResources, Deferred / Infeasible / InProgress conditions) count as CalculateResource counts
    them (framework/types.go:1035-1076 with helpers.go:193-320) in the device mirror: a stream scheduled
    on small nodes, where Fit and the allocation scores depend on those requests, matches the oracle pod by
    pod, through batches (the persistent loop) and single calls; resized pods are also removed and re-added
    between batches; the mirror equals the cache."""
    rng, cfg, nodes, existing, names = rand_cluster(4200 + seed, n_nodes=[64, 300, 700, 1100][seed], n_existing=0,
                                                    cfg_index=[0, 1, 3, 2][seed])
    for n in nodes:  # small nodes: the resized pods' requests decide Fit
        n["status"]["allocatable"]["cpu"] = rng.choice(["4", "6", "8"])
        n["status"]["allocatable"]["memory"] = rng.choice(["8Gi", "12Gi", "16Gi"])
    existing = []
    for k in range(len(nodes) * 2):
        p = add_resize_status(rng, rand_pod(rng, 300000 + k, names, topology=False))
        p["spec"].get("affinity", {}).pop("nodeAffinity", None)
        p["spec"]["nodeName"] = rng.choice(names)
        existing.append(p)
    g, o = _pair(native, cfg, nodes, existing)
    assert g.compare_mirror(sync=True) == (0, -1)
    k = 0
    for rnd in range(4):
        pods = [rand_pod(rng, 10 * k + j, names, topology=False) for j in range(60)]
        if rnd % 2:  # a few incoming pods carry status too (Fit ignores it, the scores read it)
            pods = [add_resize_status(rng, p) if rng.random() < 0.3 else p for p in pods]
        rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
        for j, p in enumerate(pods):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[j].as_tuple() == ro.as_tuple(), f"seed {seed} round {rnd} pod {j}"
        for j in range(8):  # single calls
            p = rand_pod(rng, 10 * k + 100 + j, names, topology=False)
            rg, _ = g.schedule_one(g.compile(p), assume=True)
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rg.as_tuple() == ro.as_tuple(), f"seed {seed} round {rnd} single {j}"
        for p in rng.sample(existing, 5):  # a resized pod's delete and re-add
            for b in (g, o):
                b.remove_pod(p["metadata"]["uid"])
                b.add_pod(p)
        k += 1
        assert g.compare_mirror(sync=True) == (0, -1)


def test_deferred_slots_then_pod_table_batch(native):
    """A node-local pipelined batch takes its pod-table slots in each pod's compile (after the first launch;
    the device pod_node column keeps room for them), here reusing slots freed by pod deletions; the next
    batch's pods read the pod table (PodTopologySpread / InterPodAffinity): it must see every placement of
    the first batch, and the mirror must equal the cache."""
    from ksg.synth import scheduling_basic, topology_spreading
    nodes, init, _ = topology_spreading(800, 600, 0)
    g, o = _pair(native, {}, nodes, init)
    for p in init[::3]:  # free pod-table slots for the next batch's compiles to reuse
        for b in (g, o):
            b.remove_pod(p["metadata"]["uid"])
    _, _, local = scheduling_basic(800, 0, 700)
    for k, p in enumerate(local):
        p["metadata"]["uid"] = f"local-{k}"
        p["metadata"]["name"] = f"local-{k}"
        p["metadata"]["namespace"] = "sched-1"  # the spread pods' namespace: their selector counts these
        p["metadata"].setdefault("labels", {})["color"] = "blue" if k % 2 else "green"
    rs = g.schedule_batch([g.compile(p) for p in local], assume=True)
    for k, p in enumerate(local):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"node-local pod {k}"
    _, _, spread = topology_spreading(800, 0, 300)
    for k, p in enumerate(spread):
        p["metadata"]["uid"] = f"spread-{k}"
        p["metadata"]["name"] = f"spread-{k}"
        p["spec"]["topologySpreadConstraints"][0]["labelSelector"] = {"matchLabels": {"color": "blue"}}
    rs = g.schedule_batch([g.compile(p) for p in spread], assume=True)
    for k, p in enumerate(spread):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"spread pod {k}"
    assert g.compare_mirror(sync=True) == (0, -1)


def test_ties_follow_heap_preorder(native):
    """All nodes identical: every TotalScore ties, so placement is the heap pre-order rule."""
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(1000, 0, 400)
    g, o = _pair(native, {}, nodes, init)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"pod {k}"


def test_scheduling_basic_5k_hetero(native):
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(5000, 1000, 300, hetero=True)
    g, o = _pair(native, {}, nodes, init)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"pod {k}"


@pytest.mark.parametrize("seed", range(4))
def test_plugin_entry_points(native, seed):
    rng, cfg, nodes, existing, names = rand_cluster(2000 + seed, n_nodes=97, n_existing=30)
    g, o = _pair(native, cfg, nodes, existing)
    for k in range(25):
        pod = rand_pod(rng, k, names)
        hg, ho = g.compile(pod), o.compile(pod)
        for plugin in ["NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity", "NodePorts",
                       "NodeResourcesFit", "PodTopologySpread", "InterPodAffinity"]:
            assert g.run_filter_plugin(hg, plugin) == o.run_filter_plugin(ho, plugin), f"{plugin} pod {k}"
        listed = sorted(rng.sample(range(len(names)), len(names) // 2))
        for plugin in ["TaintToleration", "NodeAffinity", "NodeResourcesFit", "PodTopologySpread", "InterPodAffinity",
                       "NodeResourcesBalancedAllocation", "ImageLocality"]:
            assert g.run_score_plugin(hg, plugin) == o.run_score_plugin(ho, plugin), f"{plugin} pod {k}"
            assert g.run_score_plugin(hg, plugin, listed) == o.run_score_plugin(ho, plugin, listed), f"{plugin} {k}"


def test_forget_and_cache_events(native):
    rng, cfg, nodes, existing, names = rand_cluster(77, n_nodes=200, n_existing=50, cfg_index=0)
    g, o = _pair(native, cfg, nodes, existing)
    handles = []
    for k in range(30):
        hg, ho, r = _cmp_cycle(g, o, rand_pod(rng, k, names), f"pod {k}")
        if r.status == 0:  # only assumed pods can be forgotten
            handles.append((hg, ho))
    for hg, ho in handles[::3]:  # Cache.ForgetPod of a third of the assumed pods
        g.forget(hg)
        o.forget(ho)
    for victim in names[5:40:7]:  # node removals re-order the snapshot
        g.remove_node(victim)
        o.remove_node(victim)
    gone = set(names[5:40:7])
    for p in [p for p in existing if p["spec"]["nodeName"] not in gone][:10]:
        g.remove_pod(p["metadata"]["uid"])
        o.remove_pod(p["metadata"]["uid"])
    upd = dict(nodes[50])
    upd["metadata"] = dict(upd["metadata"], labels={"kubernetes.io/hostname": names[50], "disk": "ssd"})
    g.update_node(upd)
    o.update_node(upd)
    for i in range(3):
        extra = dict(nodes[0])
        extra["metadata"] = {"name": f"late-{i}", "labels": {"topology.kubernetes.io/zone": "zone-c"}}
        g.add_node(extra)
        o.add_node(extra)
    assert g.node_names() == o.node_names()
    for k in range(30, 60):
        _cmp_cycle(g, o, rand_pod(rng, k, names), f"after events pod {k}")


def test_empty_cluster_and_unschedulable(native):
    g, o = _pair(native, {}, [], [])
    pod = rand_pod(random.Random(1), 0, [])
    hg, ho = g.compile(pod), o.compile(pod)
    assert g.schedule_one(hg)[0].as_tuple() == o.schedule_one(ho)[0].as_tuple()


def _stream(native, nodes, init, pods, cfg=None, ocfg=None, batch=None):
    """The pods through ksg_schedule_batch (in batches of `batch`), each assume landing before the
    next pod, against the oracle (ocfg: e.g. cpuThreads for the large clusters)."""
    g = native(dict(cfg or {}))
    o = oracle(dict(cfg or {}, **(ocfg or {})))
    for b in (g, o):
        for ns in namespaces():
            b.upsert_namespace(ns)
        for n in nodes:
            b.add_node(n)
        for p in init:
            b.add_pod(p)
    assert g.node_names() == o.node_names()
    hs = [g.compile(p) for p in pods]
    step = batch or len(pods)
    rs = []
    for i in range(0, len(hs), step):
        rs += g.schedule_batch(hs[i:i + step], assume=True)
    ors = o.schedule_batch([o.compile(p) for p in pods], assume=True)
    for k in range(len(pods)):
        assert rs[k].as_tuple() == ors[k].as_tuple(), f"pod {k}: {rs[k].as_tuple()} != oracle {ors[k].as_tuple()}"
    return rs


def test_c3_pod_affinity_1k(native):
    from ksg.synth import scheduling_pod_affinity
    _stream(native, *scheduling_pod_affinity(1000, 1000, 150))


def test_c4_topology_spreading_3k(native):
    from ksg.synth import topology_spreading
    _stream(native, *topology_spreading(3000, 3000, 150))


def test_c4_preferred_anti_affinity_2k(native):
    from ksg.synth import topology_spreading
    _stream(native, *topology_spreading(2000, 2000, 120, preferred_anti=True))


# ---- the BASELINE configs at their own sizes -----------------------------------------
def test_c3_baseline_size(native):
    """configs[2]: 5000 nodes in zone1 (1000 tainted foo:NoSchedule), 5000 pod-affinity init pods,
    pod-affinity / node-affinity / node-inclusion-policy spread pods in turn."""
    from ksg.synth import scheduling_c3
    rs = _stream(native, *scheduling_c3(5000, 5000, 240), ocfg={"cpuThreads": 16}, batch=80)
    assert sum(r.status == 0 for r in rs) == len(rs)


@pytest.mark.parametrize("anti", [False, True])
def test_c4_baseline_size(native, anti):
    """configs[3]: 15000 nodes (zones moon-1/2/3), 15000 init pods, zone spread maxSkew 5 (or
    preferred hostname anti-affinity)."""
    from ksg.synth import topology_spreading
    _stream(native, *topology_spreading(15000, 15000, 160, preferred_anti=anti), ocfg={"cpuThreads": 16}, batch=80)


def test_c5_mixed_100k(native):
    """configs[4] on one GPU: 100000 heterogeneous nodes in 10 zones (1 % tainted), 10000 bound pods,
    the mixed stream (50 % default, 10 % each node-affinity / pod-affinity / anti-affinity /
    preferred anti-affinity / zone spread)."""
    from ksg.synth import mixed_cluster
    _stream(native, *mixed_cluster(100000, 10000, 200), ocfg={"cpuThreads": 16}, batch=100)


@pytest.mark.parametrize("wg", [1, 3, 7, 64, 256])
def test_persistent_loop_geometries(native, wg):
    """k_sched_loop with 1..256 workgroups (1 -> one workgroup owns every node block) against the
    oracle: heterogeneous nodes (untied scores), then all-tied nodes (heap pre-order)."""
    from ksg.synth import scheduling_basic
    for hetero, n_nodes in ((True, 3000), (False, 1500)):
        nodes, init, pods = scheduling_basic(n_nodes, 300, 250, hetero=hetero)
        g, o = _pair(native, {"loopWorkgroups": wg}, nodes, init)
        rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
        for k, p in enumerate(pods):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[k].as_tuple() == ro.as_tuple(), f"wg {wg} hetero {hetero} pod {k}"


@pytest.mark.parametrize("wave_map", [1, 2])
def test_persistent_loop_wave_maps(native, wave_map):
    """k_sched_loop with its roles on other hardware waves (loopWaveMap): the same results as the
    oracle on heterogeneous and all-tied clusters and on a random mixed stream."""
    from ksg.synth import scheduling_basic
    for hetero, n_nodes in ((True, 3000), (False, 1500)):
        nodes, init, pods = scheduling_basic(n_nodes, 300, 300, hetero=hetero)
        g, o = _pair(native, {"loopWaveMap": wave_map}, nodes, init)
        rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
        for k, p in enumerate(pods):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[k].as_tuple() == ro.as_tuple(), f"map {wave_map} hetero {hetero} pod {k}"
    rng, cfg, nodes, existing, names = rand_cluster(5100 + wave_map, n_nodes=800, n_existing=80)
    g, o = _pair(native, dict(cfg, loopWaveMap=wave_map), nodes, existing)
    pods = [rand_pod(rng, k, names) for k in range(120)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"map {wave_map} mixed pod {k}"


@pytest.mark.parametrize("seed", range(4))
def test_persistent_loop_mixed_runs(native, seed):
    """Random pods: runs of node-local pods go through k_sched_loop, PTS/IPA pods through the
    per-pod launches, interleaved on one stream -- identical to the loop-less path and the oracle."""
    rng, cfg, nodes, existing, names = rand_cluster(5000 + seed, n_nodes=800, n_existing=80)
    g, o = _pair(native, cfg, nodes, existing)
    g2, _ = _pair(native, dict(cfg, persistentLoop=False), nodes, existing)
    pods = [rand_pod(rng, k, names) for k in range(120)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    rs2 = g2.schedule_batch([g2.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple() == rs2[k].as_tuple(), f"seed {seed} pod {k}"


@pytest.mark.parametrize("seed,wg", [(0, 0), (1, 0), (2, 1), (3, 5), (4, 0), (5, 64)])
def test_agg_loop_matches_launch_path(native, seed, wg):
    """k_agg_loop (PodTopologySpread / InterPodAffinity pods in one persistent launch): random pods
    with hostname-keyed (node-local counts) and zone / disk-keyed (shared counts) constraints and
    terms, in one batch, against the per-pod launch path (aggLoop off) and the oracle."""
    rng, cfg, nodes, existing, names = rand_cluster(7000 + seed, n_nodes=[300, 700, 1100][seed % 3], n_existing=150)
    base = dict(cfg, loopWorkgroups=wg) if wg else cfg
    g, o = _pair(native, base, nodes, existing)
    g2, _ = _pair(native, dict(base, aggLoop=False), nodes, existing)
    pods = [rand_pod(rng, k, names) for k in range(160)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    rs2 = g2.schedule_batch([g2.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple() == rs2[k].as_tuple(), f"seed {seed} pod {k}"
    assert g.compare_mirror(sync=False) == (0, -1), "device mirror differs from the cache after the batch"


@pytest.mark.parametrize("seed", range(3))
def test_agg_loop_pipelined_batch(native, seed):
    """400 random pods in one batch: chunks after the first are compiled while k_agg_loop runs, with
    every pod's slot (and its affinity terms) reserved up front -- identical to the sequential oracle
    and to the per-pod launch path, unplaced pods included."""
    rng, cfg, nodes, existing, names = rand_cluster(7100 + seed, n_nodes=[400, 900, 260][seed], n_existing=150)
    g, o = _pair(native, cfg, nodes, existing)
    g2, _ = _pair(native, dict(cfg, aggLoop=False), nodes, existing)
    pods = [rand_pod(rng, k, names) for k in range(400)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    rs2 = g2.schedule_batch([g2.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple() == rs2[k].as_tuple(), f"seed {seed} pod {k}"
    assert g.compare_mirror(sync=False) == (0, -1)


def _crowd(rng, pod, n_cons, n_terms):
    """More PodTopologySpread constraints / pod (anti-)affinity terms than k_agg_loop takes (8 per
    kind): the launch path evaluates them (the limit is 32 constraints, 64 terms per kind)."""
    from fuzz_gen import rand_label_selector, rand_pa_term, TOPO_KEYS
    spec = pod.o["spec"] if hasattr(pod, "o") else pod["spec"]
    cs = spec.setdefault("topologySpreadConstraints", [])
    for _ in range(n_cons):
        c = {"maxSkew": rng.randint(1, 12), "topologyKey": rng.choice(TOPO_KEYS),
             "whenUnsatisfiable": "DoNotSchedule" if rng.random() < 0.3 else "ScheduleAnyway"}
        sel = rand_label_selector(rng)
        if sel is not None:
            c["labelSelector"] = sel
        cs.append(c)
    if n_terms:
        aff = spec.setdefault("affinity", {})
        for kind in ("podAffinity", "podAntiAffinity"):
            a = aff.setdefault(kind, {})
            if rng.random() < 0.5:  # required terms: most select pods that do not exist (a feasible rest)
                ts = [rand_pa_term(rng) for _ in range(n_terms)]
                for t in ts:
                    if rng.random() < (0.85 if kind == "podAntiAffinity" else 0.0):
                        t["labelSelector"] = {"matchLabels": {"app": "absent"}}
                    elif kind == "podAffinity":
                        t["labelSelector"] = {}
                        t.pop("namespaceSelector", None)
                a["requiredDuringSchedulingIgnoredDuringExecution"] = ts
            a["preferredDuringSchedulingIgnoredDuringExecution"] = [
                {"weight": rng.randint(1, 100), "podAffinityTerm": rand_pa_term(rng)} for _ in range(n_terms)]
    return pod


@pytest.mark.parametrize("seed", range(3))
def test_many_constraints_and_terms(native, seed):
    """Pods with 9..32 spread constraints and 9..20 affinity terms per kind (formerly KSG_ENOTSUP):
    per-cycle results and per-node evaluations, then a pipelined batch mixing them with random pods,
    against the oracle."""
    rng, cfg, nodes, existing, names = rand_cluster(7200 + seed, n_nodes=[150, 333, 600][seed], n_existing=120)
    g, o = _pair(native, cfg, nodes, existing)
    for k in range(16):
        pod = rand_pod(rng, k, names, topology=False)
        _crowd(rng, pod.o if hasattr(pod, "o") else pod, rng.randint(9, 32) if k % 2 == 0 else rng.randint(0, 3),
               rng.randint(9, 20) if k % 4 < 2 else 0)
        _cmp_cycle(g, o, pod, f"seed {seed} pod {k}")
    pods = []
    for k in range(300):
        pod = rand_pod(rng, 100 + k, names)
        if k % 5 == 0:
            _crowd(rng, pod.o if hasattr(pod, "o") else pod, rng.randint(9, 12), rng.randint(0, 10))
        pods.append(pod)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"seed {seed} batch pod {k}"


@pytest.mark.parametrize("agg", [False, True])
def test_loop_give_up_recovers(native, agg):
    """A persistent loop that gives up (forced with debugLoopGiveUpAt: every workgroup stops at the
    6th pod of a run, as if one never arrived) fails the batch with KSG_EDEVICE and schedules none of
    its pods; the device mirror, which holds the first pods' assumes, differs from the cache until
    the next cycle rebuilds it (ksg_debug_compare_mirror), and scheduling then continues exactly as
    the oracle's, which never saw the failed batch."""
    from ksg.abi import KsgError
    from ksg.synth import scheduling_basic, topology_spreading
    nodes, init, pods = topology_spreading(600, 600, 60) if agg else scheduling_basic(600, 100, 60, hetero=True)
    g = native({"debugLoopGiveUpAt": 5})
    o = oracle({})
    for b in (g, o):
        for n in nodes:
            b.add_node(n)
        for p in init:
            b.add_pod(p)
    assert g.compare_mirror(sync=True) == (0, -1)
    hs = [g.compile(p) for p in pods[:40]]
    with pytest.raises(KsgError, match="not scheduled"):
        g.schedule_batch(hs, assume=True)
    nd, first = g.compare_mirror(sync=False)
    assert nd > 0 and first >= 0, "the device assumes of the failed run should still be in the mirror"
    assert g.compare_mirror(sync=True) == (0, -1)
    hs = [g.compile(p) for p in pods]  # the same pods again, in runs shorter than the give-up point
    rs = []
    for i in range(0, len(hs), 5):
        rs += g.schedule_batch(hs[i:i + 5], assume=True)
    ors = o.schedule_batch([o.compile(p) for p in pods], assume=True)
    for k in range(len(pods)):
        assert rs[k].as_tuple() == ors[k].as_tuple(), f"pod {k}"
    assert g.compare_mirror(sync=False) == (0, -1)


@pytest.mark.parametrize("seed", range(3))
def test_node_add_remove_by_gather(native, seed):
    """Node adds, removes and zone moves between cycles move the unchanged nodes' device columns to
    their new snapshot index (relayout_gather) instead of rebuilding the mirror: the mirror equals
    the cache after every cycle, the scheduling equals the oracle's, and the gather path is taken."""
    rng, cfg, nodes, existing, names = rand_cluster(9100 + seed, n_nodes=700, n_existing=120)
    g, o = _pair(native, cfg, nodes, existing)
    _cmp_cycle(g, o, rand_pod(rng, 0, names), "warm-up", evaluate=False)
    full0, gat0 = g.relayouts()
    k = 1
    for step in range(12):
        kind = step % 3
        if kind == 0:  # add two nodes (zones drawn as the generator does)
            for j in range(2):
                extra = dict(nodes[rng.randrange(len(nodes))])
                extra["metadata"] = dict(extra["metadata"], name=f"add-{seed}-{step}-{j}",
                                         labels=dict(extra["metadata"].get("labels", {}),
                                                     **{"kubernetes.io/hostname": f"add-{seed}-{step}-{j}"}))
                g.add_node(extra)
                o.add_node(extra)
        elif kind == 1:  # remove a node (its pods become a ghost's)
            victim = g.node_names()[rng.randrange(len(g.node_names()))]
            g.remove_node(victim)
            o.remove_node(victim)
        else:  # a zone move
            nm = g.node_names()[rng.randrange(len(g.node_names()))]
            src = next(n for n in nodes if n["metadata"]["name"] == nm) if any(
                n["metadata"]["name"] == nm for n in nodes) else None
            if src is not None:
                upd = dict(src)
                upd["metadata"] = dict(src["metadata"], labels=dict(src["metadata"].get("labels", {}),
                                                                    **{"topology.kubernetes.io/zone": "zone-b"}))
                g.update_node(upd)
                o.update_node(upd)
        for _ in range(4):
            _cmp_cycle(g, o, rand_pod(rng, k, names), f"seed {seed} step {step} pod {k}", evaluate=False)
            k += 1
        assert g.compare_mirror(sync=False) == (0, -1), f"mirror differs from the cache after step {step}"
    full1, gat1 = g.relayouts()
    assert gat1 - gat0 >= 6, f"node events re-laid out by gather only {gat1 - gat0} times (full {full1 - full0})"


# ---- percentageOfNodesToScore: the cut feasible list and the device-resident nextStartNodeIndex
# (schedule_one.go:778-884, 686-687).  Random clusters are >= 100 nodes so the cut is active; the
# no-score profile takes numNodesToFind = 1 (schedule_one.go:780-782).
NO_SCORE = {"disabledPlugins": ["TaintToleration", "NodeAffinity", "NodeResourcesFit", "PodTopologySpread",
                                "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"]}
SAMPLING = [(0, {}), (7, {}), (30, {}), (55, {"nodeResourcesFit": {"scoringStrategy": {"type": "MostAllocated"}}}),
            (0, {"interPodAffinity": {"hardPodAffinityWeight": 5}}), (100, NO_SCORE), (20, NO_SCORE)]


@pytest.mark.parametrize("k", range(len(SAMPLING)))
@pytest.mark.parametrize("seed", range(3))
def test_sampling_sequences_match_oracle(native, k, seed):
    pct, extra = SAMPLING[k]
    rng, _, nodes, existing, names = rand_cluster(5000 + 10 * k + seed, n_nodes=[130, 257, 600][seed], n_existing=60)
    cfg = dict(extra, percentageOfNodesToScore=pct)
    g, o = _pair(native, cfg, nodes, existing)
    for q in range(30):
        _cmp_cycle(g, o, rand_pod(rng, q, names), f"pct {pct} seed {seed} pod {q}")


@pytest.mark.parametrize("k", range(len(SAMPLING)))
def test_sampling_batch_matches_sequential_oracle(native, k):
    """The rotation is carried pod to pod on the device inside one batch."""
    pct, extra = SAMPLING[k]
    rng, _, nodes, existing, names = rand_cluster(6000 + k, n_nodes=700, n_existing=80)
    cfg = dict(extra, percentageOfNodesToScore=pct)
    g, o = _pair(native, cfg, nodes, existing)
    for rnd in range(2):  # two batches: the host picks the rotation up from the first
        pods = [rand_pod(rng, 400 * rnd + q, names) for q in range(300)]  # >= 256: the chunked pipeline
        rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
        for q, p in enumerate(pods):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[q].as_tuple() == ro.as_tuple(), f"pct {pct} batch {rnd} pod {q}"


def test_sampling_prefilter_subset_over_100_nodes(native):
    """A PreFilterResult (matchFields metadata.name) of 150 nodes is itself sampled: the rotation
    runs over the subset list and nextStartNodeIndex advances by the subset's processed count."""
    from ksg.objects import PodW
    rng, _, nodes, existing, names = rand_cluster(77, n_nodes=400, n_existing=40)
    g, o = _pair(native, {"percentageOfNodesToScore": 10}, nodes, existing)
    for q in range(12):
        sub = rng.sample(names, 150)
        p = PodW(f"s{q}", uid=f"s{q}").req({"cpu": "100m"}).node_affinity_required(
            [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": sub}]}]).obj()
        _cmp_cycle(g, o, p, f"subset pod {q}")
        _cmp_cycle(g, o, rand_pod(rng, q, names), f"pod {q}")


# ---- the host pipeline's fallbacks (engine.cpp run_batch): a later chunk whose compile references a
# label key no node column holds yet (mirror re-layout mid-batch), or whose programs outgrow the
# staging buffers sized from chunk 0, drains the device, mirrors the finished chunks and re-lays
# out -- the results must still be the sequential oracle's.
def _pipeline_cluster(n_nodes=900):
    from ksg.objects import NodeW
    nodes = []
    for i in range(n_nodes):
        w = NodeW(f"node-{i:05d}").capacity({"cpu": "8", "memory": "32Gi", "pods": "110"}) \
            .label("kubernetes.io/hostname", f"node-{i:05d}").label("rack", f"r{i % 7}").label("tier", f"t{i % 3}")
        for q in range(12):
            w = w.label(f"k{q}", f"v{(i + q) % 4}")
        nodes.append(w.obj())
    return nodes


def test_pipeline_relayout_mid_batch(native):
    from ksg.objects import PodW
    nodes = _pipeline_cluster()
    pods = []
    for k in range(700):
        p = PodW(f"p{k}", uid=f"p{k}").req({"cpu": "100m", "memory": "200Mi"})
        if k >= 300 and k % 5 == 0:  # first seen after chunk 0: new label columns mid-batch, more
            # than the column capacity the mirror was laid out with (a full re-layout)
            p = p.node_selector({f"k{(k // 10) % 12}": f"v{k % 4}"} if k % 2 else {"tier": f"t{k % 3}"})
        pods.append(p.obj())
    _stream(native, nodes, [], pods)


def test_pipeline_staging_outgrown_mid_batch(native):
    from ksg.objects import PodW
    nodes = _pipeline_cluster()
    pods = []
    for k in range(700):
        p = PodW(f"q{k}", uid=f"q{k}").req({"cpu": "50m", "memory": "100Mi"})
        if k >= 200:  # far larger programs than chunk 0's: many preferred node-affinity terms
            p = p.node_affinity_preferred([(1 + (j % 9), {"matchExpressions": [
                {"key": "kubernetes.io/hostname", "operator": "In",
                 "values": [f"node-{(k * 31 + j * 7 + v) % 900:05d}" for v in range(40)]}]}) for j in range(16)])
        pods.append(p.obj())
    _stream(native, nodes, [], pods)


# ---- incremental mirror ingestion: Cache.UpdateNode for a node that keeps
# its snapshot position and its taint / image counts is rewritten in place on the device
# (Cluster::upload_node_static); other updates take the full re-layout.  Both against the oracle.
@pytest.mark.parametrize("seed", range(3))
def test_node_updates_in_place(native, seed):
    import copy
    rng, cfg, nodes, existing, names = rand_cluster(900 + seed, n_nodes=[130, 300, 520][seed], n_existing=80)
    g, o = _pair(native, cfg, nodes, existing)
    cur = {n["metadata"]["name"]: n for n in nodes}
    for rnd in range(10):
        for _ in range(6):
            nm = rng.choice(names)
            n = copy.deepcopy(cur[nm])
            st, md, sp = n["status"], n["metadata"], n.setdefault("spec", {})
            r = rng.random()
            if r < 0.3:  # allocatable
                st["allocatable"]["cpu"] = rng.choice(["1", "4", "8", "16", "2500m"])
                st["allocatable"]["memory"] = rng.choice(["2Gi", "8Gi", "32Gi"])
            elif r < 0.45:
                sp["unschedulable"] = not sp.get("unschedulable", False)
            elif r < 0.65:  # label values of existing keys (zone kept: same snapshot position)
                lb = md.setdefault("labels", {})
                lb["gen"] = str(rng.randint(1, 9))
                lb["disk"] = rng.choice(["ssd", "hdd", "nvme"])
            elif r < 0.85 and sp.get("taints"):  # same taint count, other values / effects
                for t in sp["taints"]:
                    t["value"] = rng.choice(["", "x", "y", "z"])
                    t["effect"] = rng.choice(["NoSchedule", "PreferNoSchedule", "NoExecute"])
            else:  # a layout change: zone moved, or a taint added
                if rng.random() < 0.5:
                    md.setdefault("labels", {})["topology.kubernetes.io/zone"] = f"zone-x{rng.randint(0, 2)}"
                else:
                    sp.setdefault("taints", []).append({"key": "extra", "value": "", "effect": "PreferNoSchedule"})
            cur[nm] = n
            g.update_node(n)
            o.update_node(n)
        assert g.node_names() == o.node_names()
        for q in range(8):
            _cmp_cycle(g, o, rand_pod(rng, 100 * rnd + q, names), f"seed {seed} round {rnd} pod {q}")


# ---- cache churn: UpdateSnapshot keeps the snapshot list across zone
# moves until a node is added or removed (cache.go:223-290); ghost NodeInfos hold the pods of nodes
# that are not (or no longer) there (cache.go:442-446, 666-689).  Random event streams between
# scheduling cycles and batches, against the oracle (which restates the same cache rules).
@pytest.mark.parametrize("seed", range(4))
def test_cache_churn_matches_oracle(native, seed):
    import copy
    from fuzz_gen import rand_node
    rng, cfg, nodes, existing, names = rand_cluster(4400 + seed, n_nodes=[90, 260, 300, 700][seed], n_existing=50)
    g, o = _pair(native, cfg, nodes, existing)
    live = {n["metadata"]["name"]: n for n in nodes}
    gone = {}   # removed nodes (their pods may still be in the cache: ghosts)
    pods_on = {}  # uid -> node of the extra bound pods this test adds
    nxt = 10000
    both = (g, o)
    for rnd in range(12):
        for _ in range(rng.randint(2, 7)):
            r = rng.random()
            if r < 0.3 and live:  # zone move (or label change) of a live node
                nm = rng.choice(sorted(live))
                n = copy.deepcopy(live[nm])
                n["metadata"].setdefault("labels", {})["topology.kubernetes.io/zone"] = rng.choice(
                    ["zone-a", "zone-b", "zone-c", "zone-d"])
                live[nm] = n
                for b in both:
                    b.update_node(n)
            elif r < 0.45:  # a new node
                n = rand_node(rng, nxt)
                nxt += 1
                live[n["metadata"]["name"]] = n
                for b in both:
                    b.add_node(n)
            elif r < 0.6 and len(live) > 5:  # a node removed (its pods stay: a ghost)
                nm = rng.choice(sorted(live))
                gone[nm] = live.pop(nm)
                for b in both:
                    b.remove_node(nm)
            elif r < 0.7 and gone:  # a removed node comes back (maybe in another zone)
                nm = rng.choice(sorted(gone))
                n = copy.deepcopy(gone.pop(nm))
                n["metadata"].setdefault("labels", {})["topology.kubernetes.io/zone"] = rng.choice(["zone-a", "zone-e"])
                live[nm] = n
                for b in both:
                    b.add_node(n)
            elif r < 0.85:  # a bound pod, sometimes on a node the cache does not know (yet)
                p = rand_pod(rng, 50000 + nxt, names, topology=True)
                nxt += 1
                p["spec"].get("affinity", {}).pop("nodeAffinity", None)
                target = rng.choice(sorted(live) + sorted(gone) + [f"future-{rng.randint(0, 3)}"])
                p["spec"]["nodeName"] = target
                pods_on[p["metadata"]["uid"]] = target
                for b in both:
                    b.add_pod(p)
            elif pods_on:  # a pod delete event
                uid = rng.choice(sorted(pods_on))
                del pods_on[uid]
                for b in both:
                    b.remove_pod(uid)
        if rng.random() < 0.3:  # a "future" node arrives: its ghost pods join it
            nm = f"future-{rng.randint(0, 3)}"
            if nm not in live:
                n = rand_node(rng, 0)
                n["metadata"]["name"] = nm
                n["metadata"]["labels"]["kubernetes.io/hostname"] = nm
                live[nm] = n
                gone.pop(nm, None)
                for b in both:
                    b.add_node(n)
        assert g.node_names() == o.node_names(), f"seed {seed} round {rnd}: snapshot order"
        for q in range(4):
            _cmp_cycle(g, o, rand_pod(rng, 100 * rnd + q, sorted(live)), f"seed {seed} round {rnd} pod {q}")
        batch = [rand_pod(rng, 7000 + 100 * rnd + q, sorted(live), topology=False) for q in range(20)]
        rs = g.schedule_batch([g.compile(p) for p in batch], assume=True)
        for q, p in enumerate(batch):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[q].as_tuple() == ro.as_tuple(), f"seed {seed} round {rnd} batch pod {q}"


@pytest.mark.parametrize("pct", [0, 30])
def test_sampling_pipelined_batch(native, pct):
    """Default-plugin pods in 600-pod batches take the chunked pipeline; the device-resident
    nextStartNodeIndex crosses the chunks (k_sched_loop carries it from pod to pod and launch to launch)."""
    from ksg import synth
    nodes, init, pods = synth.scheduling_basic(700, 100, 1200, hetero=True)
    g, o = _pair(native, {"percentageOfNodesToScore": pct}, nodes, init)
    for rnd in range(2):
        part = pods[600 * rnd:600 * (rnd + 1)]
        rs = g.schedule_batch([g.compile(p) for p in part], assume=True)
        for q, p in enumerate(part):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[q].as_tuple() == ro.as_tuple(), f"pct {pct} batch {rnd} pod {q}"


@pytest.mark.parametrize("unit,n_nodes", [(128, 5000), (256, 5000), (128, 300), (128, 1100)])
def test_sched_loop_units_match_oracle(native, unit, n_nodes):
    """k_sched_loop with 128-node workgroups (two evaluation waves) and with 256-node ones: SchedulingBasic
    (every score tied: the heap pre-order rule across workgroups) and random node-local pods."""
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(n_nodes, n_nodes // 5, 300, hetero=n_nodes != 5000)
    g, o = _pair(native, {"loopUnit": unit}, nodes, init)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    assert g.kernel_stats()[3] == "k_sched_loop"
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"pod {k}"
    rng, cfg, nodes, existing, names = rand_cluster(9100 + n_nodes, n_nodes=n_nodes if n_nodes < 5000 else 700,
                                                    n_existing=100, topology=False)
    g, o = _pair(native, dict(cfg, loopUnit=unit), nodes, existing)
    pods = [rand_pod(rng, k, names, topology=False) for k in range(200)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"random pod {k}"
    assert g.compare_mirror(sync=False) == (0, -1)


@pytest.mark.parametrize("unit", [128, 256])
def test_sched_loop_prepared_and_fixup_paths(native, unit):
    """k_sched_loop installs the chosen node's next evaluation prepared before the winner is known
    (default-plugin pods) or has the owner re-evaluate it (a host-port pod after a host-port pod, a
    node-affinity pod): runs that alternate the two, with every score tied and untied, must match the
    oracle pod by pod."""
    from ksg.objects import PodW
    from ksg.synth import scheduling_basic
    for hetero in (True, False):
        nodes, init, base = scheduling_basic(1500, 200, 180, hetero=hetero)
        g, o = _pair(native, {"loopUnit": unit}, nodes, init)
        pods = []
        for k, p in enumerate(base):
            if k % 7 in (3, 4):  # two host-port pods in a row: the second cannot be prepared
                p = PodW(f"hp{k}", uid=f"hp{k}").container(requests={"cpu": "100m"}).host_port(8000 + k % 5).obj()
            elif k % 11 == 5:
                p = PodW(f"na{k}", uid=f"na{k}").container(requests={"cpu": "200m"}).node_affinity_in(
                    "kubernetes.io/hostname", [nodes[j]["metadata"]["name"] for j in range(k % 9, 1500, 13)]).obj()
            pods.append(p)
        rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
        assert g.kernel_stats()[3] == "k_sched_loop"
        for k, p in enumerate(pods):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[k].as_tuple() == ro.as_tuple(), f"unit {unit} hetero {hetero} pod {k}"
        assert g.compare_mirror(sync=False) == (0, -1)


@pytest.mark.parametrize("relay", [False, True])
def test_resident_single_pod_calls(native, relay):
    """ksg_schedule_one through the resident loop (node-local pods) against the oracle, pod by pod, with
    the events that must stop it in between: informer events, a forget, a batch, pods it declines
    (PodTopologySpread), an idle gap longer than its self-stop, and more calls than one launch holds;
    relay: workgroup 0 relays the doorbell through device memory (ringRelayMinWorkgroups 1, the path of
    clusters with many workgroups)."""
    import time
    rng, cfg, nodes, existing, names = rand_cluster(9300, n_nodes=900, n_existing=90, topology=False)
    g, o = _pair(native, dict(cfg, ringRelayMinWorkgroups=1) if relay else cfg, nodes, existing)
    hist = []

    def one(pod, tag):
        rg, _ = g.schedule_one(g.compile(pod), assume=True)
        ro, _ = o.schedule_one(o.compile(pod), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"{tag}: {rg.as_tuple()} != {ro.as_tuple()}"
        hist.append(pod)

    for k in range(60):
        one(rand_pod(rng, k, names, topology=False), f"pod {k}")
    # informer events between calls
    extra = rand_cluster(9301, n_nodes=12, n_existing=0, topology=False)[2]
    for n in extra:
        n["metadata"]["name"] += "-late"
        n["metadata"].setdefault("labels", {})["kubernetes.io/hostname"] = n["metadata"]["name"]
        for b in (g, o):
            b.add_node(n)
    names = g.node_names()
    for k in range(60, 120):
        one(rand_pod(rng, k, names, topology=False), f"pod {k} (after node adds)")
    # forget, then a pod the loop declines, then a batch
    hg, ho = g.compile(hist[-1]), o.compile(hist[-1])
    rg, _ = g.schedule_one(hg, assume=True)
    ro, _ = o.schedule_one(ho, assume=True)
    assert rg.as_tuple() == ro.as_tuple()
    g.forget(hg)
    o.forget(ho)
    for k in range(120, 160):
        one(rand_pod(rng, k, names), f"pod {k} (mixed, some declined)")
    batch = [rand_pod(rng, 1000 + k, names, topology=False) for k in range(30)]
    rs = g.schedule_batch([g.compile(p) for p in batch], assume=True)
    for k, p in enumerate(batch):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"batch pod {k}"
    time.sleep(0.08)  # longer than the loop's idle self-stop
    for k in range(160, 1300):  # past one launch's kLoopMaxPods
        one(rand_pod(rng, k, names, topology=False), f"pod {k}")
    assert g.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("seed", range(2))
def test_resident_agg_single_pod_calls(native, seed):
    """ksg_schedule_one of PodTopologySpread / InterPodAffinity pods through the resident k_agg_loop (the
    pod's program and its pod-table entry through the ring; the owner of the chosen node writes the entry
    and appends the pod, so the next calls count it), mixed with node-local pods and Service-selected pods
    (system default spreading), with informer events, a forget, batches and an idle gap in between, and
    more calls than one launch holds -- pod by pod against the oracle, the mirror against the cache."""
    import time
    from fuzz_gen import rand_objects
    rng, cfg, nodes, existing, names = rand_cluster(9500 + seed, n_nodes=[700, 1500][seed], n_existing=150)
    g, o = _pair(native, cfg, nodes, existing)
    for ob in rand_objects(rng):
        for b in (g, o):
            b.upsert_object(ob)
    agg = 0

    def one(pod, tag):
        nonlocal agg
        rg, _ = g.schedule_one(g.compile(pod), assume=True)
        ro, _ = o.schedule_one(o.compile(pod), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"{tag}: {rg.as_tuple()} != {ro.as_tuple()}"
        agg += g.kernel_stats()[3] == "k_agg_loop"
        return pod

    hist = [one(rand_pod(rng, k, names), f"pod {k}") for k in range(200)]
    extra = rand_cluster(9510 + seed, n_nodes=10, n_existing=0)[2]
    for n in extra:  # informer events between calls: node adds, a bound pod, a pod deleted
        n["metadata"]["name"] += "-late"
        n["metadata"].setdefault("labels", {})["kubernetes.io/hostname"] = n["metadata"]["name"]
        for b in (g, o):
            b.add_node(n)
    names = g.node_names()
    bound = rand_pod(rng, 5000, names)
    bound["spec"]["nodeName"] = names[7]
    for b in (g, o):
        b.add_pod(bound)
        b.remove_pod(existing[3]["metadata"]["uid"])
    hist += [one(rand_pod(rng, k, names), f"pod {k} (after events)") for k in range(200, 400)]
    for p in reversed(hist):  # a forget (of a pod that gets placed again)
        hg, ho = g.compile(p), o.compile(p)
        rg, _ = g.schedule_one(hg, assume=True)
        ro, _ = o.schedule_one(ho, assume=True)
        assert rg.as_tuple() == ro.as_tuple()
        if rg.status == 0:
            g.forget(hg)
            o.forget(ho)
            break
    batch = [rand_pod(rng, 2000 + k, names) for k in range(40)]
    rs = g.schedule_batch([g.compile(p) for p in batch], assume=True)
    for k, p in enumerate(batch):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"batch pod {k}"
    time.sleep(0.08)  # longer than the loop's idle self-stop
    for k in range(400, 1300):  # past one launch's kLoopMaxPods
        one(rand_pod(rng, k, names, topology=k % 3 != 0), f"pod {k}")
    assert agg > 600, f"only {agg} calls ran in the resident k_agg_loop"
    assert g.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("unit", [128, 256])
@pytest.mark.parametrize("k", [0, 1, 2, 3, 5, 6])
def test_sched_loop_sampling_matches_oracle(native, unit, k):
    """percentageOfNodesToScore inside k_sched_loop: the cut to the first K feasible nodes of the rotated
    order, processedNodes from the (K+1)-th node's workgroup, nextStartNodeIndex carried pod to pod, the
    kept-list maxima exchange (PreferNoSchedule taints, preferred node affinity), and runs broken by
    launch-path pods (PodTopologySpread / InterPodAffinity) that read the loop's rotation and back."""
    pct, extra = SAMPLING[k]
    for seed, (n_nodes, topo) in enumerate([(700, False), (1900, True), (5000, False)]):
        rng, cfg, nodes, existing, names = rand_cluster(9400 + 10 * k + seed, n_nodes=n_nodes, n_existing=120,
                                                        topology=topo)
        # (the no-score profile disables PodTopologySpread, so OpportunisticBatching would act and its signed
        # pods take the launch path: the gate is off here, this test is about the loop)
        g, o = _pair(native, dict(cfg, **extra, percentageOfNodesToScore=pct, loopUnit=unit,
                                  featureGates={"OpportunisticBatching": False}), nodes, existing)
        for rnd in range(2):
            pods = [rand_pod(rng, 500 * rnd + q, names, topology=topo and q % 5 == 2) for q in range(150)]
            rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
            if not topo:
                assert g.kernel_stats()[3] == "k_sched_loop"
            for q, p in enumerate(pods):
                ro, _ = o.schedule_one(o.compile(p), assume=True)
                assert rs[q].as_tuple() == ro.as_tuple(), f"pct {pct} nodes {n_nodes} batch {rnd} pod {q}"
        assert g.compare_mirror(sync=False) == (0, -1)


def test_sched_loop_sampling_scheduling_basic(native):
    """SchedulingBasic at upstream's adaptive default (percentageOfNodesToScore 0: 10 % of 5000 nodes)
    through k_sched_loop, every score tied: the heap pre-order over the cut list and the rotation."""
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(5000, 1000, 1200)
    g, o = _pair(native, {"percentageOfNodesToScore": 0}, nodes, init)
    for rnd in range(2):
        part = pods[600 * rnd:600 * (rnd + 1)]
        rs = g.schedule_batch([g.compile(p) for p in part], assume=True)
        assert g.kernel_stats()[3] == "k_sched_loop"
        for q, p in enumerate(part):
            ro, _ = o.schedule_one(o.compile(p), assume=True)
            assert rs[q].as_tuple() == ro.as_tuple(), f"batch {rnd} pod {q}"


@pytest.mark.parametrize("pct", [0, 30])
def test_resident_single_pod_calls_sampling(native, pct):
    """The resident loop with percentageOfNodesToScore: each call's rotation start is the host's
    nextStartNodeIndex, which the call's result (processedNodes) advances; batches in between."""
    rng, cfg, nodes, existing, names = rand_cluster(9320 + pct, n_nodes=1300, n_existing=90, topology=False)
    g, o = _pair(native, dict(cfg, percentageOfNodesToScore=pct), nodes, existing)
    for k in range(200):
        pod = rand_pod(rng, k, names, topology=False)
        rg, _ = g.schedule_one(g.compile(pod), assume=True)
        ro, _ = o.schedule_one(o.compile(pod), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"pod {k}: {rg.as_tuple()} != {ro.as_tuple()}"
        if k % 50 == 49:
            batch = [rand_pod(rng, 1000 + k * 10 + j, names, topology=False) for j in range(20)]
            rs = g.schedule_batch([g.compile(p) for p in batch], assume=True)
            for j, p in enumerate(batch):
                ro, _ = o.schedule_one(o.compile(p), assume=True)
                assert rs[j].as_tuple() == ro.as_tuple(), f"batch after pod {k}, pod {j}"
    assert g.compare_mirror(sync=True)[0] == 0


def test_resident_loop_off_matches(native):
    """residentLoop false: the same calls take the launch path (results identical)."""
    rng, cfg, nodes, existing, names = rand_cluster(9310, n_nodes=500, n_existing=50, topology=False)
    g, o = _pair(native, dict(cfg, residentLoop=False), nodes, existing)
    for k in range(40):
        pod = rand_pod(rng, k, names, topology=False)
        rg, _ = g.schedule_one(g.compile(pod), assume=True)
        ro, _ = o.schedule_one(o.compile(pod), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"pod {k}"


@pytest.mark.parametrize("wg", [0, 7])
def test_agg_loop_same_template_runs(native, wg):
    """Runs of identical pods (one template: DF_AGG_SAME, no gather -- the previous pod's counts plus its
    placement) broken by pods of other templates, on zoned nodes with bound pods: topology spreading
    (DoNotSchedule zone minima recomputed after each fold), preferred / required anti-affinity, required
    affinity, and unplaceable pods (the fold adds nothing).  Against the oracle and the loop with the
    shortcut off (aggLoopDebug 4)."""
    from ksg import synth
    nodes, init, _ = synth.topology_spreading(900, 600, 0)
    kinds = [synth.pod_with_topology_spreading, synth.pod_with_preferred_pod_anti_affinity,
             synth.pod_with_required_anti_affinity, synth.pod_with_pod_affinity]
    pods, k = [], 0
    for run, kind in enumerate([0, 0, 1, 0, 2, 1, 1, 3, 0, 2, 0, 1]):
        for _ in range([30, 1, 12, 45, 3, 20][run % 6]):
            pods.append(kinds[kind](f"t{k}", "sched-1"))
            k += 1
    big = synth.pod_with_topology_spreading("huge", "sched-1")
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "1000"}}
    pods[40:40] = [big, dict(big, metadata=dict(big["metadata"], name="huge2", uid="huge2"))]
    base = {"loopWorkgroups": wg} if wg else {}
    g, o = _pair(native, base, nodes, init)
    g2, _ = _pair(native, dict(base, aggLoopDebug=4), nodes, init)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    rs2 = g2.schedule_batch([g2.compile(p) for p in pods], assume=True)
    assert g.kernel_stats()[3] == "k_agg_loop"
    for q, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[q].as_tuple() == ro.as_tuple() == rs2[q].as_tuple(), f"pod {q} ({p['metadata']['name']})"
    assert g.compare_mirror(sync=False) == (0, -1)


@pytest.mark.parametrize("wg,seed", [(0, 0), (7, 1), (1, 2), (0, 3)])
def test_agg_loop_template_cache(native, wg, seed):
    """k_agg_loop's template cache: pods of up to nine templates in random order (more than the six slots, so
    templates are evicted and gathered again), C3's rotation among them -- pod affinity, node affinity beside
    existing affinity terms, hostname spread honouring node affinity and taints (node-local DoNotSchedule minima:
    the counts are kept or loaded, exchange Z after the placement) -- zone spread, required / preferred
    anti-affinity, unplaceable pods.  A pod of a cached template loads its counts and folds the previous pod's
    placement in; every placement is folded into the other cached templates.  Against the oracle and the loop
    with the cache off (aggLoopDebug 32)."""
    from ksg import synth
    rng = random.Random(8800 + seed)
    nodes, init, _ = synth.scheduling_c3(700, 500, 0)
    for k, n in enumerate(nodes):  # two zones, so zone spread and zone affinity have more than one domain
        n["metadata"]["labels"]["topology.kubernetes.io/zone"] = f"zone{1 + k % 2}"
    kinds = [lambda n: synth.pod_with_pod_affinity(n, "sched-1"),
             lambda n: synth.pod_with_node_affinity(n, "sched-1", ["zone1", "zone2"]),
             lambda n: synth.pod_with_node_inclusion_policy(n, "sched-1"),
             lambda n: synth.pod_with_topology_spreading(n, "sched-1"),
             lambda n: synth.pod_with_required_anti_affinity(n, "sched-1"),
             lambda n: synth.pod_with_preferred_pod_anti_affinity(n, "sched-1"),
             lambda n: synth.pod_with_node_affinity(n, "sched-1", ["zone2"]),
             lambda n: synth.pod_with_pod_affinity(n, "sched-0"),
             lambda n: synth.pod_with_topology_spreading(n, "sched-0")]
    pods = []
    for k in range(360):
        if k < 90:
            kind = k % 3  # C3's rotation first
        else:
            kind = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 2, 2, 0])
        pods.append(kinds[kind](f"c{k}"))
    big = synth.pod_with_node_inclusion_policy("huge", "sched-1")
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "1000"}}
    pods[120:120] = [big]
    base = {"loopWorkgroups": wg} if wg else {}
    g, o = _pair(native, base, nodes, init)
    g2, _ = _pair(native, dict(base, aggLoopDebug=32), nodes, init)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    rs2 = g2.schedule_batch([g2.compile(p) for p in pods], assume=True)
    assert g.kernel_stats()[3] == "k_agg_loop"
    for q, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[q].as_tuple() == ro.as_tuple() == rs2[q].as_tuple(), f"pod {q} ({p['metadata']['name']})"
    assert g.compare_mirror(sync=False) == (0, -1)


@pytest.mark.parametrize("debug", [0, 8, 28, -1])
def test_resident_agg_same_template_calls(native, debug):
    """ksg_schedule_one of runs of identical pods through the resident k_agg_loop: a pod posted right after
    one of its template is not staged over PCIe (RING_SAME: the loop copies the previous program and
    entry in LDS and patches slot, rotation and label offset) and starts from the counts the loop folded
    at the end of the previous pod (DF_AGG_SAME).  Spread pods (zone DoNotSchedule), pods with own
    affinity terms (no fold, entries differ), unplaceable pods (nothing to fold), Service-selected pods
    under system default spreading (their PodTopologySpread raw scores computed in phase 1 with the
    previous pod's topology sizes, exchange PX skipped when the sizes hold); against the oracle pod by pod,
    with the shortcuts off (aggLoopDebug 8: every pod staged; 28: staged, gathered, PX always), and the
    mirror against the cache."""
    from ksg import synth
    nodes, init, _ = synth.topology_spreading(900, 600, 0)
    dnodes, dinit, dpods, objects = synth.default_topology_spreading(0, 0, 40)
    kinds = [synth.pod_with_topology_spreading, synth.pod_with_preferred_pod_anti_affinity,
             synth.pod_with_required_anti_affinity, synth.pod_with_pod_affinity]
    pods, k = [], 0
    for run, kind in enumerate([0, 0, 1, 0, 2, 1, 1, 3, 0, 2, 0, 1]):
        for _ in range([30, 1, 12, 45, 3, 20][run % 6]):
            pods.append(kinds[kind](f"t{k}", "sched-1"))
            k += 1
    big = synth.pod_with_topology_spreading("huge", "sched-1")
    big["spec"]["containers"][0]["resources"] = {"requests": {"cpu": "1000"}}
    pods[40:40] = [big, dict(big, metadata=dict(big["metadata"], name="huge2", uid="huge2"))]
    pods[100:100] = dpods
    # (debug -1: the doorbell and the staged program relayed through device memory, ringRelayMinWorkgroups 1)
    g, o = _pair(native, {"ringRelayMinWorkgroups": 1} if debug < 0 else {"aggLoopDebug": debug} if debug else {},
                 nodes, init)
    for ob in objects:
        for b in (g, o):
            b.upsert_object(ob)
    agg = 0
    for q, p in enumerate(pods):
        rg, _ = g.schedule_one(g.compile(p), assume=True)
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"pod {q} ({p['metadata']['name']})"
        agg += g.kernel_stats()[3] == "k_agg_loop"
    assert agg > len(pods) * 3 // 4, f"only {agg} of {len(pods)} calls ran in the resident k_agg_loop"
    assert g.compare_mirror(sync=True)[0] == 0


def test_resident_ring_same_flag_only_difference(native):
    """ksg_schedule_one of consecutive pods whose programs differ in one flag bit only (DF_TERMINATING: every
    third pod carries a deletionTimestamp, so as an assumed pod it counts for nobody's spreading): the resident
    k_agg_loop's RING_SAME shortcut reuses the previous program with the slot, rotation and DF_AGG_SAME patched,
    so it must not take such a pod for the same one.  Against the oracle pod by pod, and the
    mirror against the cache."""
    from ksg import synth
    nodes, init, _ = synth.topology_spreading(900, 600, 0)
    g, o = _pair(native, {}, nodes, init)
    agg = 0
    for k in range(45):
        p = synth.pod_with_topology_spreading(f"f{k}", "sched-1")
        if k % 3 == 1:
            p["metadata"]["deletionTimestamp"] = "2024-01-01T00:00:00Z"
        rg, _ = g.schedule_one(g.compile(p), assume=True)
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"pod {k}"
        agg += g.kernel_stats()[3] == "k_agg_loop"
    assert agg > 30, f"only {agg} of 45 calls ran in the resident k_agg_loop"
    assert g.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("wg", [1, 0])
def test_agg_loop_spilled_lists(native, wg):
    """k_agg_loop workgroups whose nodes hold more pods / affinity terms than their LDS lists (5120 each in
    the batch loop, 2048 in the resident one): the rest go to HBM spill rows (AggView::spill).  500 zoned
    nodes with 8500 bound pods, 5500 of them carrying a preferred anti-affinity term, then a mixed PTS / IPA
    batch -- one workgroup (wg 1) or the default geometry -- against the oracle and the per-pod launch path,
    then single-pod calls through the resident loop against the oracle."""
    from ksg import synth
    nodes, init, pods = synth.mixed_cluster(500, 3000, 260)
    names = [n["metadata"]["name"] for n in nodes]
    for k in range(5500):
        p = synth.pod_with_preferred_pod_anti_affinity(f"pa-{k}", "sched-1")
        p["spec"]["nodeName"] = names[(k * 7) % len(names)]
        init.append(p)
    base = {"loopWorkgroups": wg} if wg else {}
    g, o = _pair(native, base, nodes, init)
    g2, _ = _pair(native, dict(base, aggLoop=False), nodes, init)
    batch, single = pods[:200], pods[200:]
    rs = g.schedule_batch([g.compile(p) for p in batch], assume=True)
    assert g.kernel_stats()[3] == "k_agg_loop"
    rs2 = g2.schedule_batch([g2.compile(p) for p in batch], assume=True)
    for q, p in enumerate(batch):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[q].as_tuple() == ro.as_tuple() == rs2[q].as_tuple(), f"pod {q} ({p['metadata']['name']})"
    assert g.compare_mirror(sync=False) == (0, -1)
    agg = 0
    for q, p in enumerate(single):
        rg, _ = g.schedule_one(g.compile(p), assume=True)
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rg.as_tuple() == ro.as_tuple(), f"single pod {q} ({p['metadata']['name']})"
        agg += g.kernel_stats()[3] == "k_agg_loop"
    assert agg > len(single) // 2
    assert g.compare_mirror(sync=True)[0] == 0

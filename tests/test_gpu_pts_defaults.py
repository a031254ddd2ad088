"""PodTopologySpread default constraints on the device against the oracle.

Pods without constraints of their own get the profile's default constraints with the selector
helper.DefaultSelector builds from the Services / RCs / ReplicaSets / StatefulSets selecting them
(podtopologyspread/common.go:59-75, plugins/helper/spread.go:37-95).  Under System defaulting the
score runs with requireAllTopologies = false: no node is ignored and a node without the zone label
is in the "" zone (scoring.go:141-144, 61-115).  Bit-exact bar as test_gpu_parity.py.
"""
import random

import pytest

from fuzz_gen import PTS_DEFAULT_CONFIGS, add_owner, namespaces, rand_cluster, rand_objects, rand_pod
from oracle_binding import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from ksg.native import Scheduler
    return Scheduler


def _pair(native, cfg, nodes, existing, objects):
    bs = []
    for make in (native, oracle):
        b = make(cfg)
        for ns in namespaces():
            b.upsert_namespace(ns)
        for o in objects:
            b.upsert_object(o)
        for n in nodes:
            b.add_node(n)
        for p in existing:
            b.add_pod(p)
        bs.append(b)
    assert bs[0].node_names() == bs[1].node_names()
    return bs


def _owned_pod(rng, k, names, own_rate=0.2):
    p = rand_pod(rng, k, names, topology=rng.random() < own_rate)
    return add_owner(rng, p)


@pytest.mark.parametrize("seed", range(16))
def test_default_constraints_match_oracle(native, seed):
    cfg = dict(PTS_DEFAULT_CONFIGS[seed % len(PTS_DEFAULT_CONFIGS)])
    rng, _, nodes, existing, names = rand_cluster(5000 + seed, n_nodes=[40, 130, 257, 300][seed % 4], n_existing=80)
    objects = rand_objects(rng)
    g, o = _pair(native, cfg, nodes, existing, objects)
    for k in range(40):
        pod = _owned_pod(rng, k, names)
        hg, ho = g.compile(pod), o.compile(pod)
        rg, eg = g.schedule_one(hg, assume=True, evaluate=True)
        ro, eo = o.schedule_one(ho, assume=True, evaluate=True)
        assert rg.as_tuple() == ro.as_tuple(), f"seed {seed} pod {k}: {rg.as_tuple()} != {ro.as_tuple()}"
        for key in eo:
            assert eg[key] == eo[key], f"seed {seed} pod {k}: eval[{key}] differs"
        if k % 13 == 12:  # object churn: the next pods see the listers' new state
            victim = objects.pop(rng.randrange(len(objects)))
            md = victim["metadata"]
            for b in (g, o):
                b.remove_object(victim["kind"], md["namespace"], md["name"])


@pytest.mark.parametrize("seed", range(4))
def test_default_constraints_batch_matches_sequential_oracle(native, seed):
    cfg = dict(PTS_DEFAULT_CONFIGS[seed % len(PTS_DEFAULT_CONFIGS)])
    rng, _, nodes, existing, names = rand_cluster(6000 + seed, n_nodes=700, n_existing=300, topology=False)
    objects = rand_objects(rng, 12)
    g, o = _pair(native, cfg, nodes, existing, objects)
    pods = [_owned_pod(rng, k, names, own_rate=0.1) for k in range(200)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"seed {seed} pod {k}"


def test_default_topology_spreading_workload(native):
    """scheduler_perf DefaultTopologySpreading (topology_spreading/performance-config.yaml:102-147) at
    1000 nodes: zones moon-1..3, one Service selecting app=scheduler-perf in service-ns."""
    from ksg.synth import default_topology_spreading
    nodes, init, pods, objects = default_topology_spreading(1000, 1000, 500)
    g, o = _pair(native, {}, nodes, init, objects)
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    assert g.kernel_stats()[3] == "k_agg_loop"  # the system-default scoring runs in the persistent loop
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple(), f"pod {k}"


@pytest.mark.parametrize("seed", range(3))
def test_default_constraints_plugin_entry_points(native, seed):
    cfg = dict(PTS_DEFAULT_CONFIGS[seed % len(PTS_DEFAULT_CONFIGS)])
    rng, _, nodes, existing, names = rand_cluster(7000 + seed, n_nodes=97, n_existing=40)
    objects = rand_objects(rng)
    g, o = _pair(native, cfg, nodes, existing, objects)
    for k in range(20):
        pod = _owned_pod(rng, k, names)
        hg, ho = g.compile(pod), o.compile(pod)
        assert g.run_filter_plugin(hg, "PodTopologySpread") == o.run_filter_plugin(ho, "PodTopologySpread"), k
        listed = sorted(rng.sample(range(len(names)), len(names) // 2))
        assert g.run_score_plugin(hg, "PodTopologySpread") == o.run_score_plugin(ho, "PodTopologySpread"), k
        assert g.run_score_plugin(hg, "PodTopologySpread", listed) == o.run_score_plugin(ho, "PodTopologySpread",
                                                                                         listed), k


def _soft_pod(rng, k, names):
    """A pod whose PodTopologySpread work is scoring only: ScheduleAnyway constraints of its own (on zone,
    hostname or disk, some with inclusion policies), or none (then the system defaults apply)."""
    from fuzz_gen import rand_label_selector, TOPO_KEYS
    p = add_owner(rng, rand_pod(rng, k, names, topology=False))
    if rng.random() < 0.5:
        cs = []
        for key in rng.sample(TOPO_KEYS, rng.randint(1, 2)):
            c = {"maxSkew": rng.randint(1, 6), "topologyKey": key, "whenUnsatisfiable": "ScheduleAnyway"}
            sel = rand_label_selector(rng)
            if sel is not None:
                c["labelSelector"] = sel
            if rng.random() < 0.2:
                c["nodeTaintsPolicy"] = "Honor"
            cs.append(c)
        p["spec"]["topologySpreadConstraints"] = cs
    return p


@pytest.mark.parametrize("seed,wg", [(0, 0), (1, 3), (2, 0), (3, 17)])
def test_agg_loop_pts_scoring_matches_launch_path(native, seed, wg):
    """PodTopologySpread scoring inside k_agg_loop (counts per node in LDS, topology sizes from exchange
    A's presence bits, NormalizeScore over exchange PX) against the per-pod launch path and the oracle."""
    rng, _, nodes, existing, names = rand_cluster(8000 + seed, n_nodes=[300, 700, 1100, 520][seed], n_existing=200)
    objects = rand_objects(rng, 12)
    cfg = {"loopWorkgroups": wg} if wg else {}
    g, o = _pair(native, cfg, nodes, existing, objects)
    g2, _ = _pair(native, dict(cfg, aggLoop=False), nodes, existing, objects)
    pods = [_soft_pod(rng, k, names) for k in range(160)]
    rs = g.schedule_batch([g.compile(p) for p in pods], assume=True)
    assert g.kernel_stats()[3] == "k_agg_loop"
    rs2 = g2.schedule_batch([g2.compile(p) for p in pods], assume=True)
    for k, p in enumerate(pods):
        ro, _ = o.schedule_one(o.compile(p), assume=True)
        assert rs[k].as_tuple() == ro.as_tuple() == rs2[k].as_tuple(), f"seed {seed} pod {k}"
    assert g.compare_mirror(sync=False) == (0, -1)

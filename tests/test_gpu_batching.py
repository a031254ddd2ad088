"""OpportunisticBatching on the device (k_ob_hint / k_ob_store) against the oracle's
restatement of framework/runtime/batch.go, pod by pod: hints taken and refused (signature changes, the
500 ms maxBatchAge, a last chosen node that is not full, a hinted node that fails), the heap's pop order,
percentageOfNodesToScore, node adds / removes between calls, evaluation output and forgets."""
import random

import pytest

from fuzz_gen import namespaces, rand_cluster, rand_pod
from oracle_binding import oracle

pytestmark = pytest.mark.gpu

NO_TOPOLOGY = {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}}


def _pair(cfg, nodes, existing=()):
    from ksg.native import Scheduler
    bs = []
    for make in (Scheduler, oracle):
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


def _hinted(r):
    return r.status == 0 and r.evaluated_nodes == 1 and r.feasible_nodes == 1


@pytest.mark.parametrize("kind", ["hostport", "saturation"])
@pytest.mark.parametrize("mode", ["batch", "calls"])
def test_batching_workloads_match_oracle(kind, mode):
    """HostPortConflict / ResourceSaturation (scheduler_perf batching/performance-config.yaml) with the
    no-topology profile: more pods than nodes, so the stream ends in FitErrors."""
    from ksg.synth import batching
    nodes, pods = batching(300, 360, kind)
    g, o = _pair(NO_TOPOLOGY, nodes)
    for b in (g, o):
        b.set_clock(10 ** 15)
    if mode == "batch":
        rg = [r.as_tuple() for r in g.schedule_batch([g.compile(p) for p in pods], assume=True)]
    else:
        rg = [g.schedule_one(g.compile(p), assume=True)[0].as_tuple() for p in pods]
    ro = [o.schedule_one(o.compile(p), assume=True)[0] for p in pods]
    for k in range(len(pods)):
        assert rg[k] == ro[k].as_tuple(), f"pod {k}: {rg[k]} != oracle {ro[k].as_tuple()}"
    hinted, cycles = g.batching()
    assert hinted == sum(_hinted(r) for r in ro) and hinted > 250, hinted
    assert cycles == len(pods)
    assert g.compare_mirror(sync=True) == (0, -1)


def _stream_pods(rng, names, n):
    """Signed templates of both kinds (one pod per node / many per node), and unsigned pods between them."""
    from ksg.objects import PodW
    out = []
    tmpl = 0
    for k in range(n):
        if rng.random() < 0.15:
            tmpl = rng.randrange(5)
        if tmpl == 0:  # HostPortConflict's pod: one per node
            p = PodW(f"hp-{k}", "default").container(image="registry.k8s.io/pause:3.10.1",
                                                      requests={"cpu": "100m", "memory": "100Mi"},
                                                      ports=[{"containerPort": 80, "hostPort": 80}])
        elif tmpl == 1:  # a big pod: about one per node
            p = PodW(f"big-{k}", "prod").container(image="registry.example/app:v1",
                                                    requests={"cpu": "2500m", "memory": "3Gi"})
        elif tmpl == 2:  # small pods: the last chosen node is not full
            p = PodW(f"small-{k}", "dev").container(image="registry.example/db", requests={"cpu": "100m"})
        elif tmpl == 3:  # a random pod (mostly unsigned: spread constraints / pod affinity, or unique labels)
            out.append(rand_pod(rng, 9000 + k, names))
            continue
        else:  # hostPort pods with a toleration and a preferred node affinity (a different signature)
            p = PodW(f"hpt-{k}", "default").container(image="registry.k8s.io/pause:3.10.1",
                                                       requests={"cpu": "200m"},
                                                       ports=[{"containerPort": 8080, "hostPort": 8080}])
            p.tolerations([{"key": "dedicated", "operator": "Exists"}])
            p.node_affinity_preferred([(5, {"matchExpressions": [{"key": "disk", "operator": "In",
                                                                  "values": ["ssd"]}]})])
        out.append(p.obj())
    return out


@pytest.mark.parametrize("seed", range(6))
def test_random_streams_match_oracle(seed):
    """Random clusters and profiles (List without defaults, or PodTopologySpread disabled; sometimes
    percentageOfNodesToScore 0) with template runs, batches and single calls, a clock that sometimes jumps
    past maxBatchAge, node adds / removes and forgets between calls."""
    rng, cfg, nodes, existing, names = rand_cluster(8800 + seed, n_nodes=[40, 130, 300, 520, 260, 90][seed],
                                                    n_existing=30, cfg_index=seed % 3)
    cfg = dict(cfg)
    if seed % 2:
        cfg["disabledPlugins"] = list(cfg.get("disabledPlugins", [])) + ["PodTopologySpread"]
    else:
        cfg.update(NO_TOPOLOGY)
    if seed in (2, 5):
        cfg["percentageOfNodesToScore"] = 0
    g, o = _pair(cfg, nodes, existing)
    t = 10 ** 15
    placed = {}
    for rnd in range(8):
        pods = _stream_pods(rng, names, rng.choice([1, 1, 3, 40, 120]))
        t += rng.choice([10 ** 6, 10 ** 7, 6 * 10 ** 8])  # sometimes past maxBatchAge
        for b in (g, o):
            b.set_clock(t)
        hg = [g.compile(p) for p in pods]
        if len(pods) > 1 and rng.random() < 0.6:
            rg = [r.as_tuple() for r in g.schedule_batch(hg, assume=True)]
        else:
            rg = [g.schedule_one(h, assume=True)[0].as_tuple() for h in hg]
        for k, p in enumerate(pods):
            ho = o.compile(p)
            ro = o.schedule_one(ho, assume=True)[0].as_tuple()
            assert rg[k] == ro, f"seed {seed} round {rnd} pod {k}: {rg[k]} != oracle {ro}"
            if ro[0] == 0:
                placed[(rnd, k)] = (hg[k], ho)
        ev = rng.random()
        if ev < 0.3 and placed:  # a binding failed: ForgetPod
            key = rng.choice(sorted(placed))
            hg_, ho_ = placed.pop(key)
            g.forget(hg_)
            o.forget(ho_)
        elif ev < 0.5:  # a node joins (the node list is rebuilt: stored indices move)
            from fuzz_gen import rand_node
            n = rand_node(rng, 50000 + rnd)
            for b in (g, o):
                b.add_node(n)
        elif ev < 0.6 and len(names) > 5:  # a node leaves
            nm = names.pop(rng.randrange(len(names)))
            for b in (g, o):
                b.remove_node(nm)
        assert g.node_names() == o.node_names()
    assert g.compare_mirror(sync=True) == (0, -1)


def test_eval_output_of_hinted_pods():
    """A hinted cycle evaluates one node: no statuses, no scores (the oracle's evaluation output agrees)."""
    from ksg.synth import batching
    nodes, pods = batching(120, 40, "hostport")
    g, o = _pair(NO_TOPOLOGY, nodes)
    for b in (g, o):
        b.set_clock(10 ** 15)
    hinted = 0
    for k, p in enumerate(pods):
        rg, eg = g.schedule_one(g.compile(p), assume=True, evaluate=True)
        ro, eo = o.schedule_one(o.compile(p), assume=True, evaluate=True)
        assert rg.as_tuple() == ro.as_tuple(), k
        assert eg == eo, f"pod {k}: evaluation output differs"
        hinted += _hinted(ro)
    assert hinted > 30


def test_gate_off_and_default_profile_run_full_cycles():
    from ksg.synth import batching
    nodes, pods = batching(150, 80, "saturation")
    for cfg in (dict(NO_TOPOLOGY, featureGates={"OpportunisticBatching": False}), {}):
        g, o = _pair(cfg, nodes)
        rg = [r.as_tuple() for r in g.schedule_batch([g.compile(p) for p in pods], assume=True)]
        ro = [o.schedule_one(o.compile(p), assume=True)[0].as_tuple() for p in pods]
        assert rg == ro
        assert g.batching()[0] == 0


def test_sharded_context_refuses_an_acting_profile():
    from ksg.abi import KsgError
    from ksg.native import Scheduler
    with pytest.raises(KsgError, match="OpportunisticBatching"):
        Scheduler(dict(NO_TOPOLOGY, device=0, distributed={"worldSize": 2, "rank": 0, "localGroup": "ob-refuse"}))


@pytest.mark.parametrize("step_ms", [0, 120, 300, 700])
def test_clock_advancing_inside_a_batch(step_ms):
    """Each scheduling cycle reads the clock (batch.go:202), not each call: with a fixed clock that advances by
    step_ms per cycle (ksg_debug_clock_step) inside one schedule_batch call, the device's hint decisions
    (maxBatchAge expiry included) equal the oracle's pod by pod."""
    from ksg.synth import batching
    nodes, pods = batching(200, 240, "hostport")
    g, o = _pair(NO_TOPOLOGY, nodes)
    for b in (g, o):
        b.set_clock(10 ** 15)
        b.clock_step(step_ms * 10 ** 6)
    rg = [r.as_tuple() for r in g.schedule_batch([g.compile(p) for p in pods], assume=True)]
    ro = [r.as_tuple() for r in o.schedule_batch([o.compile(p) for p in pods], assume=True)]
    assert rg == ro
    hinted = sum(r[2] == 1 and r[3] == 1 and r[0] == 0 for r in ro)
    assert g.batching() == (hinted, len(pods))
    if step_ms >= 500:
        assert hinted == 0
    elif step_ms == 300:
        assert 0 < hinted < len(pods) * 2 // 3

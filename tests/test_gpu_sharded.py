"""Node-sharded evaluation on the device, against the CPU oracle.

W scheduler contexts on ONE GPU form an in-process exchange group ("localGroup"): each holds
the whole cluster mirror, evaluates its contiguous range of the snapshot order, and exchanges
counts / NormalizeScore maxima / best keys through the same stream-ordered all-reduce slots the
RCCL transport uses (comm.hpp); with deviceExchange (the RCCL ranks' default, opt-in here), the
loop-eligible pods exchange through the persistent loop's granules stored into every rank's array.  Every rank must return the
oracle's ScheduleResult for every pod of the stream (sequential assume semantics), including
empty shards (clusters smaller than W * 256 nodes) and PodTopologySpread/InterPodAffinity pods.
"""
import os
import threading
import uuid

import pytest

from fuzz_gen import namespaces, rand_cluster, rand_pod
from oracle_binding import oracle

pytestmark = pytest.mark.gpu


def _group(world, cfg, nodes, existing):
    from ksg.native import Scheduler
    name = f"t-{uuid.uuid4().hex[:8]}"
    # a node-sharded scheduler does not run OpportunisticBatching (ksg_create refuses a profile where it acts,
    # e.g. PodTopologySpread disabled): the gate is off for every rank and the oracle alike
    cfg = dict(cfg)
    cfg.setdefault("featureGates", {"OpportunisticBatching": False})
    ranks = []
    for r in range(world):
        s = Scheduler(dict(cfg, device=0, distributed={"worldSize": world, "rank": r, "localGroup": name}))
        for ns in namespaces():
            s.upsert_namespace(ns)
        for n in nodes:
            s.add_node(n)
        for p in existing:
            s.add_pod(p)
        ranks.append(s)
    o = oracle(cfg)
    for ns in namespaces():
        o.upsert_namespace(ns)
    for n in nodes:
        o.add_node(n)
    for p in existing:
        o.add_pod(p)
    for s in ranks:
        assert s.node_names() == o.node_names()
    return ranks, o


def _run_ranks(ranks, pods, chunk):
    """schedule_batch on every rank concurrently (one thread per rank, as the exchange needs)."""
    hs = [[s.compile(p) for p in pods] for s in ranks]
    out = [[] for _ in ranks]
    errs = []

    def work(r):
        try:
            for k in range(0, len(pods), chunk):
                out[r].extend(x.as_tuple() for x in ranks[r].schedule_batch(hs[r][k:k + chunk], assume=True))
        except Exception as e:  # surfaced below
            errs.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(len(ranks))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    if errs:  # the whole text: a loop give-up names the missing participants per rank
        pytest.fail("\n".join(f"rank {r}: {e}" for r, e in errs), pytrace=False)
    return out


def _check(ranks, o, pods, chunk=64, forced_give_up=False):
    got = _run_ranks(ranks, pods, chunk)
    bad = []  # every rank's mismatches (the first 12), so an intermittent one is characterised when it shows
    for k, p in enumerate(pods):
        want = o.schedule_one(o.compile(p), assume=True)[0].as_tuple()
        bad += [f"rank {r} pod {k}: {got[r][k]} != oracle {want}" for r in range(len(ranks)) if got[r][k] != want]
    assert not bad, f"{len(bad)} mismatches (status, node, evaluated, feasible, score): " + "; ".join(bad[:12])
    # (give-ups, all-reduce re-runs) per rank: a recovered give-up must not pass as a clean run
    stats = [s.loop_stats() for s in ranks]
    if forced_give_up:
        assert all(g >= 1 and r >= 1 for g, r in stats), stats
    else:
        assert all(st == (0, 0) for st in stats), f"persistent-loop give-ups / re-runs per rank: {stats}"


def test_shard_ranges_partition_the_snapshot():
    from ksg.synth import scheduling_basic
    nodes, _, _ = scheduling_basic(1300, 0, 0)
    ranks, _ = _group(3, {}, nodes, [])
    spans = [s.shard_range() for s in ranks]
    assert spans[0][0] == 0
    for (a, n), (b, _) in zip(spans, spans[1:]):
        assert a + n == b and a % 256 == 0
    assert spans[-1][0] + spans[-1][1] == 1300


@pytest.mark.parametrize("world,seed", [(2, 0), (2, 1), (3, 2), (4, 3), (8, 4), (2, 5)])
def test_random_streams_match_oracle(world, seed):
    rng, cfg, nodes, existing, names = rand_cluster(3000 + seed, n_nodes=[700, 1100, 900, 1300, 2100, 600][seed],
                                                    n_existing=120)
    ranks, o = _group(world, cfg, nodes, existing)
    _check(ranks, o, [rand_pod(rng, k, names) for k in range(80)], chunk=32)


@pytest.mark.parametrize("world,seed", [(2, 0), (3, 2)])
def test_random_streams_match_oracle_device_exchange(world, seed):
    """deviceExchange on (the RCCL ranks' default): loop-eligible pods exchange through granules."""
    rng, cfg, nodes, existing, names = rand_cluster(3000 + seed, n_nodes=[700, 1100, 900][seed], n_existing=120)
    ranks, o = _group(world, dict(cfg, deviceExchange=True), nodes, existing)
    _check(ranks, o, [rand_pod(rng, k, names) for k in range(80)], chunk=32)


@pytest.mark.parametrize("world", [2, 3, 4, 6, 8])
def test_device_exchange_loop_c2(world):
    """The persistent loop across W ranks (granules stored into every rank's array), SchedulingBasic
    pods only, heterogeneous nodes (untied scores), batches long enough for the chunked pipeline.
    In-process groups launch every rank's loop in one dispatch, so any W up to
    kMaxShards runs the loop, with zero give-ups (_check)."""
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(600 * world + 77, 300, 600, hetero=True)
    ranks, o = _group(world, {"deviceExchange": True}, nodes, init)
    _check(ranks, o, pods, chunk=300)
    assert _dominant(ranks) == {"k_sched_loop"}


@pytest.mark.parametrize("world", [2, 4])
def test_small_cluster_with_empty_shards(world):
    rng, cfg, nodes, existing, names = rand_cluster(41, n_nodes=130, n_existing=30)
    ranks, o = _group(world, cfg, nodes, existing)
    _check(ranks, o, [rand_pod(rng, k, names) for k in range(40)])


def test_ties_follow_heap_preorder_across_shards():
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(2000, 0, 300)
    ranks, o = _group(4, {}, nodes, init)
    _check(ranks, o, pods, chunk=100)


def test_c4_topology_spreading_sharded():
    from ksg.synth import topology_spreading
    nodes, init, pods = topology_spreading(2000, 2000, 100)
    ranks, o = _group(2, {}, nodes, init)
    _check(ranks, o, pods, chunk=50)


def test_c4_preferred_anti_affinity_sharded():
    from ksg.synth import topology_spreading
    nodes, init, pods = topology_spreading(1500, 1500, 80, preferred_anti=True)
    ranks, o = _group(3, {}, nodes, init)
    _check(ranks, o, pods, chunk=40)


def test_c3_pod_affinity_sharded():
    from ksg.synth import scheduling_pod_affinity
    nodes, init, pods = scheduling_pod_affinity(1000, 1000, 100)
    ranks, o = _group(2, {}, nodes, init)
    _check(ranks, o, pods, chunk=50)


@pytest.mark.parametrize("world,seed", [(2, 7), (3, 8)])
def test_eval_output_gathered_when_sharded(world, seed):
    """Per-node evaluation output on a node-sharded context (the plugin-level hook's input): every rank
    returns the whole snapshot's statuses, per-plugin scores and TotalScores, gathered over the ranks,
    equal to the oracle's, for a stream of pods with assume."""
    rng, cfg, nodes, existing, names = rand_cluster(seed, n_nodes=[0, 0, 0, 0, 0, 0, 0, 700, 900][seed],
                                                    n_existing=60)
    ranks, o = _group(world, cfg, nodes, existing)
    pods = [rand_pod(rng, k, names) for k in range(25)]
    out = [[] for _ in ranks]
    errs = []

    def work(r):
        try:
            for p in pods:
                res, ev = ranks[r].schedule_one(ranks[r].compile(p), assume=True, evaluate=True)
                out[r].append((res.as_tuple(), ev))
        except Exception as e:  # surfaced below
            errs.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    for k, p in enumerate(pods):
        res, ev = o.schedule_one(o.compile(p), assume=True, evaluate=True)
        for r in range(world):
            assert out[r][k][0] == res.as_tuple(), f"rank {r} pod {k}"
            assert out[r][k][1] == ev, f"rank {r} pod {k}: evaluation output differs"


# ---- percentageOfNodesToScore on node-sharded contexts: the cut takes one more all-reduce of the
# per-rank feasible counts (k_sample_shard_a/b), the rank holding the (K+1)-th feasible node of the
# rotated order publishes end and processedNodes, and nextStartNodeIndex advances on every rank
# from them (schedule_one.go:686-687,778-884).
SHARD_SAMPLING = [(0, {}), (7, {}), (30, {}), (55, {"nodeResourcesFit": {"scoringStrategy": {"type": "MostAllocated"}}}),
                  (100, {"disabledPlugins": ["TaintToleration", "NodeAffinity", "NodeResourcesFit", "PodTopologySpread",
                                             "InterPodAffinity", "NodeResourcesBalancedAllocation", "ImageLocality"]})]


@pytest.mark.parametrize("k", range(len(SHARD_SAMPLING)))
@pytest.mark.parametrize("world", [2, 3])
def test_sampling_sharded_matches_oracle(world, k):
    pct, extra = SHARD_SAMPLING[k]
    rng, cfg, nodes, existing, names = rand_cluster(7100 + 10 * k + world, n_nodes=[0, 0, 900, 1300][world],
                                                    n_existing=80)
    ranks, o = _group(world, dict(cfg, **extra, percentageOfNodesToScore=pct), nodes, existing)
    _check(ranks, o, [rand_pod(rng, q, names) for q in range(120)], chunk=40)


def test_sampling_sharded_basic_rotation():
    """SchedulingBasic with pct 10 on W = 4: every pod's cut ends on some rank and the rotation walks
    across all four shards."""
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(2300, 200, 300, hetero=True)
    ranks, o = _group(4, {"percentageOfNodesToScore": 10}, nodes, init)
    _check(ranks, o, pods, chunk=150)


def test_sampling_sharded_with_empty_shard():
    """400 nodes (two 256-node blocks) on W = 3: one rank holds no node; the cut's counts, intervals
    and processedNodes still agree on every rank."""
    rng, cfg, nodes, existing, names = rand_cluster(7400, n_nodes=400, n_existing=40)
    ranks, o = _group(3, dict(cfg, percentageOfNodesToScore=30), nodes, existing)
    _check(ranks, o, [rand_pod(rng, q, names) for q in range(60)], chunk=20)


@pytest.mark.parametrize("world", [2, 3])
def test_sampling_sharded_eval_and_subset(world):
    """Evaluation output of a cut list (unprocessed nodes carry no status) and PreFilterResult subsets
    that are themselves sampled, gathered over the ranks."""
    from ksg.objects import PodW
    rng, cfg, nodes, existing, names = rand_cluster(7300 + world, n_nodes=1000, n_existing=60)
    ranks, o = _group(world, {"percentageOfNodesToScore": 12}, nodes, existing)
    pods = []
    for q in range(14):
        sub = rng.sample(names, 400)
        pods.append(PodW(f"s{q}", uid=f"s{q}").req({"cpu": "100m"}).node_affinity_required(
            [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": sub}]}]).obj())
        pods.append(rand_pod(rng, q, names))
    out = [[] for _ in ranks]
    errs = []

    def work(r):
        try:
            for p in pods:
                res, ev = ranks[r].schedule_one(ranks[r].compile(p), assume=True, evaluate=True)
                out[r].append((res.as_tuple(), ev))
        except Exception as e:  # surfaced below
            errs.append((r, e))

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not errs, errs
    for q, p in enumerate(pods):
        res, ev = o.schedule_one(o.compile(p), assume=True, evaluate=True)
        for r in range(world):
            assert out[r][q][0] == res.as_tuple(), f"rank {r} pod {q}"
            assert out[r][q][1] == ev, f"rank {r} pod {q}: evaluation output differs"


def test_preemption_on_sharded_ranks():
    """DefaultPreemption on a node-sharded group: each rank holds the whole mirror and runs the PostFilter
    over every node itself; every rank's choice equals the oracle's."""
    from test_gpu_preempt import build, cluster, mk_pod
    rng, nodes, existing = cluster(21, 300, 6)
    name = f"t-{uuid.uuid4().hex[:8]}"
    from ksg.native import Scheduler
    ranks = []
    for r in range(2):
        s = Scheduler({"device": 0, "distributed": {"worldSize": 2, "rank": r, "localGroup": name}})
        for ns in ("default", "team"):
            s.upsert_namespace({"metadata": {"name": ns}})
        for n in nodes:
            s.add_node(n)
        for p in existing:
            s.add_pod(p)
        ranks.append(s)
    o = build(oracle, nodes, existing)
    for q in range(8):
        pod = mk_pod(f"pre{q}", rng, prio=1000, big=True)
        args = {"offset": q * 31, "now": 1704153600 * 10 ** 9, "listCandidates": True}
        r0, d0 = o.preempt(o.compile(pod), args)
        for s in ranks:
            r1, d1 = s.preempt(s.compile(pod), args)
            assert r1.as_tuple() == r0.as_tuple() and d1 == d0, f"pod {q}"


def test_rccl_transport_single_rank_matches_oracle():
    """The RCCL transport itself (ncclGetUniqueId -> ncclCommInitRank -> in-stream ncclAllReduce
    MAX between the kernels) at worldSize 1 -- the one-GPU box cannot host two RCCL ranks."""
    from ksg.native import Scheduler, comm_unique_id
    rng, cfg, nodes, existing, names = rand_cluster(4242, n_nodes=900, n_existing=80)
    s = Scheduler(dict(cfg, device=0, distributed={"worldSize": 1, "rank": 0, "ncclId": comm_unique_id()}))
    o = oracle(cfg)
    for b in (s, o):
        for ns in namespaces():
            b.upsert_namespace(ns)
        for n in nodes:
            b.add_node(n)
        for p in existing:
            b.add_pod(p)
    pods = [rand_pod(rng, k, names) for k in range(80)]
    got = [r.as_tuple() for r in s.schedule_batch([s.compile(p) for p in pods], assume=True)]
    for k, p in enumerate(pods):
        assert got[k] == o.schedule_one(o.compile(p), assume=True)[0].as_tuple(), f"pod {k}"


@pytest.mark.parametrize("world", [2, 4, 8])
def test_c5_mixed_sharded_20k(world):
    """configs[4]'s mixed stream on 20000 nodes split over W in-process ranks (the 8-GPU layout of
    the 100k-node config, scaled to one device), against the oracle."""
    from ksg.synth import mixed_cluster
    nodes, init, pods = mixed_cluster(20000, 2000, 120)
    ranks, o = _group(world, {}, nodes, init)
    _check(ranks, o, pods, chunk=60)


# ---- k_agg_loop across ranks (deviceExchange): PodTopologySpread / InterPodAffinity pods through the
# persistent loop, granules and shared-key partials stored into every rank's arrays

def _dominant(ranks):
    return {s.kernel_stats()[3] for s in ranks}


@pytest.mark.parametrize("world", [2, 3])
def test_c5_mixed_sharded_agg_loop(world):
    """configs[4]'s mixed stream (node-local, spread and affinity pods) on 20000 nodes over W in-process
    ranks with the device exchange: the spread / affinity pods run in the node-sharded k_agg_loop."""
    from ksg.synth import mixed_cluster
    nodes, init, pods = mixed_cluster(20000, 2000, 240)
    ranks, o = _group(world, {"deviceExchange": True}, nodes, init)
    _check(ranks, o, pods, chunk=120)
    for s in ranks:
        assert s.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("world", [2, 3])
def test_c4_sharded_agg_loop(world):
    from ksg.synth import topology_spreading
    nodes, init, pods = topology_spreading(2000 * world, 2000, 300)
    ranks, o = _group(world, {"deviceExchange": True}, nodes, init)
    _check(ranks, o, pods, chunk=300)
    assert _dominant(ranks) == {"k_agg_loop"}


def test_c4_anti_sharded_agg_loop():
    from ksg.synth import topology_spreading
    nodes, init, pods = topology_spreading(3000, 3000, 200, preferred_anti=True)
    ranks, o = _group(3, {"deviceExchange": True}, nodes, init)
    _check(ranks, o, pods, chunk=200)
    assert _dominant(ranks) == {"k_agg_loop"}


def test_c3_sharded_agg_loop():
    from ksg.synth import scheduling_pod_affinity
    nodes, init, pods = scheduling_pod_affinity(2000, 2000, 300)
    ranks, o = _group(2, {"deviceExchange": True}, nodes, init)
    _check(ranks, o, pods, chunk=300)
    assert _dominant(ranks) == {"k_agg_loop"}
    for s in ranks:
        assert s.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("world,seed", [(2, 5), (3, 6)])
def test_random_streams_sharded_agg_loop(world, seed):
    """Random PodTopologySpread / InterPodAffinity pods (zone- and hostname-keyed constraints and terms,
    preferred terms, existing pods' terms) across ranks, mixed with node-local pods in one batch."""
    rng, cfg, nodes, existing, names = rand_cluster(3100 + seed, n_nodes=1400 if seed == 5 else 1700,
                                                    n_existing=200)
    ranks, o = _group(world, dict(cfg, deviceExchange=True), nodes, existing)
    _check(ranks, o, [rand_pod(rng, k, names) for k in range(200)], chunk=100)
    for s in ranks:
        assert s.compare_mirror(sync=True)[0] == 0


def test_spilled_lists_sharded_agg_loop():
    """Node-sharded k_agg_loop whose workgroups hold more pods / terms than their LDS lists (the HBM spill
    rows): 1000 zoned nodes over 2 ranks, one workgroup each, 9000 bound pods of which
    4500 carry a preferred anti-affinity term, then a mixed PTS / IPA stream."""
    from ksg import synth
    nodes, init, pods = synth.mixed_cluster(1000, 4500, 160)
    names = [n["metadata"]["name"] for n in nodes]
    for k in range(4500):
        p = synth.pod_with_preferred_pod_anti_affinity(f"pa-{k}", "sched-1")
        p["spec"]["nodeName"] = names[(k * 7) % len(names)]
        init.append(p)
    ranks, o = _group(2, {"deviceExchange": True, "loopWorkgroups": 1}, nodes, init)
    _check(ranks, o, pods, chunk=160)
    assert _dominant(ranks) == {"k_agg_loop"}
    for s in ranks:
        assert s.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("world", [2, 3])
def test_c5_pipelined_batches_sharded_agg_loop(world):
    """600-pod batches of the mixed stream over W in-process ranks with the device exchange: the batch runs
    as pipelined chunks (later chunks compiled while the loop runs, drains when staging grows), every
    rank passing the host gate before each loop launch that follows a drain."""
    from ksg.synth import mixed_cluster
    nodes, init, pods = mixed_cluster(6000, 1200, 1200)
    ranks, o = _group(world, {"deviceExchange": True}, nodes, init)
    _check(ranks, o, pods, chunk=600)
    for s in ranks:
        assert s.compare_mirror(sync=True)[0] == 0


@pytest.mark.parametrize("world", [2, 3])
def test_loop_give_up_retried_over_allreduce(world):
    """An in-process group whose persistent loops give up (forced: debugLoopGiveUpAt makes every workgroup of
    every rank stop at the same pod) re-runs the pods from the failed chunk over the all-reduce path
    (Engine::run_batch_api), every rank in step: results equal to the oracle's, mirrors equal to the caches."""
    from ksg.synth import mixed_cluster
    nodes, init, pods = mixed_cluster(3000, 600, 400)
    ranks, o = _group(world, {"deviceExchange": True, "debugLoopGiveUpAt": 40}, nodes, init)
    _check(ranks, o, pods, chunk=400, forced_give_up=True)
    for s in ranks:
        assert s.compare_mirror(sync=True)[0] == 0


def test_group_loops_start_together_after_contexts_closed():
    """The sequence that gave up in round 5: a W = 6 group beside another live context, then
    -- both closed -- a second W = 6 group, then a W = 8 group beside three live contexts.  The loops of
    separate dispatches on separate hardware queues were not co-scheduled (the give-up records showed one
    rank's loop entering only when its peers gave up, 10 s later); every group now runs its ranks' loops in
    ONE dispatch, so every group runs the loop with zero give-ups and the oracle's results."""
    from ksg.native import Scheduler
    from ksg.synth import scheduling_basic
    for world, others in ((6, 1), (6, 0), (8, 3)):
        nodes, init, pods = scheduling_basic(1877 + 256 * world, 300, 600, hetero=True)
        live = [Scheduler({"device": 0}) for _ in range(others)]
        ranks, o = _group(world, {"deviceExchange": True}, nodes, init)
        _check(ranks, o, pods, chunk=300)
        assert _dominant(ranks) == {"k_sched_loop"}
        for s in ranks + live:
            s.close()

"""evaluateNominatedNode on the device (k_nominated) against the oracle, pod by pod:
a pod whose status.nominatedNodeName names a snapshot node tries that node alone first (schedule_one.go:657-669,
714-745) and takes it when it passes (EvaluatedNodes 1, nextStartNodeIndex unchanged); otherwise that node's
status joins NodeToStatus and the full pass follows (the node counts once in EvaluatedNodes / processedNodes).

The stream the reference produces it in is DefaultPreemption's: PostFilter nominates a node, the caller deletes
the victims and patches status.nominatedNodeName, and the pod's next cycle goes there (ksg_preempt then
ksg_schedule_*).  Also random streams with nominations that pass, fail, name unknown nodes, sit outside a
PreFilterResult list or behind the percentageOfNodesToScore cut, with evaluation output, OpportunisticBatching
and the resident single-pod path."""

import pytest

from fuzz_gen import namespaces, rand_cluster, rand_pod
from oracle_binding import oracle
from test_gpu_preempt import build, cluster, mk_pod

pytestmark = pytest.mark.gpu


def _nominate(pod, node):
    pod = dict(pod)
    pod["status"] = dict(pod.get("status") or {}, nominatedNodeName=node)
    return pod


@pytest.mark.parametrize("seed", range(3))
def test_preempt_nominate_reschedule(seed):
    """preempt -> victims deleted -> nominatedNodeName set -> the pod's next cycle, on both backends."""
    from ksg.native import Scheduler
    rng, nodes, existing = cluster(100 + seed, 40 + 20 * seed, 8)
    dev, orc = build(Scheduler, nodes, existing), build(oracle, nodes, existing)
    placed = 0
    for q in range(60):  # big pods fill the cluster; the ones that no longer fit preempt
        pod = mk_pod(f"pre{q}", rng, prio=rng.choice([500, 1000]), big=True)
        rd = dev.schedule_one(dev.compile(pod), assume=True)[0].as_tuple()
        ro = orc.schedule_one(orc.compile(pod), assume=True)[0].as_tuple()
        assert rd == ro, (q, rd, ro)
        if rd[0] == 0:
            continue
        args = {"offset": rng.randrange(1000), "now": 1704067200 * 10 ** 9}
        pd, dd = dev.preempt(dev.compile(pod), args)
        po, do = orc.preempt(orc.compile(pod), args)
        assert pd.as_tuple() == po.as_tuple() and dd == do, q
        if pd.status != 0:
            continue
        for uid in dd["victims"]:
            dev.remove_pod(uid)
            orc.remove_pod(uid)
        node = dev.node_names()[pd.node_index]
        npod = _nominate(pod, node)
        rd = dev.schedule_one(dev.compile(npod), assume=True)[0].as_tuple()
        ro = orc.schedule_one(orc.compile(npod), assume=True)[0].as_tuple()
        assert rd == ro, (q, rd, ro)
        assert rd[1] == pd.node_index and rd[2] == 1 and rd[3] == 1, rd  # the nominated node alone
        placed += 1
    assert placed >= 2, placed
    assert dev.compare_mirror(sync=True) == (0, -1)


def _stream(rng, names, n):
    pods = []
    for k in range(n):
        p = rand_pod(rng, k, names)
        r = rng.random()
        if r < 0.25:
            p = _nominate(p, rng.choice(names))
        elif r < 0.3:
            p = _nominate(p, "no-such-node")
        pods.append(p)
    return pods


@pytest.mark.parametrize("pct,mode", [(100, "batch"), (100, "calls"), (30, "batch"), (0, "calls"), (100, "eval")])
def test_random_nominations_match_oracle(pct, mode):
    from ksg.native import Scheduler
    rng, cfg, nodes, existing, names = rand_cluster(5150 + pct + len(mode), n_nodes=700, n_existing=150)
    cfg = dict(cfg, percentageOfNodesToScore=pct)
    g, o = Scheduler(cfg), oracle(cfg)
    for b in (g, o):
        for ns in namespaces():
            b.upsert_namespace(ns)
        for nd in nodes:
            b.add_node(nd)
        for p in existing:
            b.add_pod(p)
    pods = _stream(rng, names, 160)
    if mode == "batch":
        got = [r.as_tuple() for r in g.schedule_batch([g.compile(p) for p in pods], assume=True)]
        for k, p in enumerate(pods):
            want = o.schedule_one(o.compile(p), assume=True)[0].as_tuple()
            assert got[k] == want, f"pod {k}: {got[k]} != oracle {want}"
    else:
        for k, p in enumerate(pods):
            if mode == "eval":
                rg, eg = g.schedule_one(g.compile(p), assume=True, evaluate=True)
                ro, eo = o.schedule_one(o.compile(p), assume=True, evaluate=True)
                assert eg == eo, f"pod {k}: evaluation output differs"
            else:
                rg = g.schedule_one(g.compile(p), assume=True)[0]
                ro = o.schedule_one(o.compile(p), assume=True)[0]
            assert rg.as_tuple() == ro.as_tuple(), f"pod {k}: {rg.as_tuple()} != oracle {ro.as_tuple()}"
    assert g.compare_mirror(sync=True) == (0, -1)


def test_nominated_outside_prefilter_result_and_signed_pods():
    """A nominated node outside the pod's PreFilterResult list (NodeAffinity matchFields) that fails alone counts
    once more; a signed OpportunisticBatching pod placed on its nominated node drops the batch state (StoreSchedule-
    Results with a nil list); evaluation output carries the failed nominated node's status."""
    from ksg.native import Scheduler
    from ksg.objects import PodW
    cfg = {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}}
    rng, _, nodes, existing, names = rand_cluster(77, n_nodes=300, n_existing=40)
    g, o = Scheduler(cfg), oracle(cfg)
    for b in (g, o):
        for ns in namespaces():
            b.upsert_namespace(ns)
        for nd in nodes:
            b.add_node(nd)
        for p in existing:
            b.add_pod(p)
        b.set_clock(10 ** 15)
    pods = []
    for q in range(40):
        sub = rng.sample(names, 30)
        p = PodW(f"s{q}", uid=f"s{q}").req({"cpu": "100m"}).node_affinity_required(
            [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": sub}]}]).obj()
        pods.append(_nominate(p, rng.choice(names)))
        big = PodW(f"b{q}", uid=f"b{q}").req({"cpu": "1500m", "memory": "1Gi"}).obj()
        pods.append(_nominate(big, rng.choice(names)) if q % 2 else big)
    for k, p in enumerate(pods):
        rg, eg = g.schedule_one(g.compile(p), assume=True, evaluate=True)
        ro, eo = o.schedule_one(o.compile(p), assume=True, evaluate=True)
        assert rg.as_tuple() == ro.as_tuple(), f"pod {k}: {rg.as_tuple()} != oracle {ro.as_tuple()}"
        assert eg == eo, f"pod {k}: evaluation output differs"
    assert g.batching()[1] == len(pods)


def test_sharded_context_declines_nominated_pods():
    from ksg.native import Scheduler
    from ksg.abi import KsgError
    import uuid
    name = f"t-{uuid.uuid4().hex[:8]}"
    ranks = [Scheduler({"device": 0, "featureGates": {"OpportunisticBatching": False},
                        "distributed": {"worldSize": 2, "rank": r, "localGroup": name}}) for r in range(2)]
    pod = _nominate({"metadata": {"name": "p", "uid": "p"}, "spec": {"containers": []}}, "n1")
    with pytest.raises(KsgError, match="rc=-5"):
        ranks[0].compile(pod)


def test_nominator_boundary_matches_oracle():
    """Other pods' nominations (ksg_add_nominated_pod): the device refuses exactly the calls the oracle refuses
    and schedules the rest identically (tests/nominator_scenario.py)."""
    from ksg.native import Scheduler
    from nominator_scenario import run
    assert run(Scheduler({})) == run(oracle({}))

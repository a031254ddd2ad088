"""The oracle's CPU-baseline mode (Filter / Score over nodes on a thread pool, as the reference's
Parallelizer.Until with 16 goroutines) gives exactly the sequential oracle's results: every
pod's result tuple and per-node evaluation output, over random clusters with every plugin.
bench.py times this mode as the multi-core CPU baseline, so it must be the same algorithm."""
import pytest

from fuzz_gen import namespaces, rand_cluster, rand_pod
from oracle_binding import oracle


def _build(cfg, nodes, existing):
    b = oracle(cfg)
    for ns in namespaces():
        b.upsert_namespace(ns)
    for n in nodes:
        b.add_node(n)
    for p in existing:
        b.add_pod(p)
    return b


@pytest.mark.parametrize("seed,threads,pw", [(0, 2, False), (1, 4, True), (2, 16, False), (3, 3, True), (4, 16, True),
                                             (5, 7, False)])
def test_parallel_oracle_matches_sequential(seed, threads, pw):
    """pw: NormalizeScore and the weights on the pool too (cpuParallelWeights)."""
    rng, cfg, nodes, existing, names = rand_cluster(seed, n_nodes=150 + 37 * seed, n_existing=60)
    seq = _build(cfg, nodes, existing)
    par = _build(dict(cfg, cpuThreads=threads, cpuParallelWeights=pw, cpuSpinUs=0 if seed % 2 else 50), nodes, existing)
    try:
        for k in range(40):
            pod = rand_pod(rng, k, names)
            rs, es = seq.schedule_one(seq.compile(pod), assume=True, evaluate=True)
            rp, ep = par.schedule_one(par.compile(pod), assume=True, evaluate=True)
            assert rs.as_tuple() == rp.as_tuple(), f"pod {k}"
            for key in es:
                assert es[key] == ep[key], f"pod {k}: eval[{key}]"
    finally:
        seq.close()
        par.close()


def test_parallel_oracle_batch_c2_shape():
    from ksg.synth import scheduling_basic
    nodes, init, pods = scheduling_basic(600, 100, 150, hetero=True)
    seq = _build({}, nodes, init)
    par = _build({"cpuThreads": 16, "cpuParallelWeights": True}, nodes, init)
    try:
        a = seq.schedule_batch([seq.compile(p) for p in pods], assume=True)
        b = par.schedule_batch([par.compile(p) for p in pods], assume=True)
        assert [r.as_tuple() for r in a] == [r.as_tuple() for r in b]
    finally:
        seq.close()
        par.close()


@pytest.mark.parametrize("seed", range(3))
def test_parallel_aggregations_match_sequential(seed):
    """The PodTopologySpread / InterPodAffinity PreFilter and PreScore aggregations on the pool (chunk-local
    counts summed, as the reference's Parallelizer passes at podtopologyspread/filtering.go:292,
    scoring.go:190, interpodaffinity/filtering.go:231,275, scoring.go:209), with Service-selected pods
    (system default spreading) and many existing pods: the sequential oracle's results and evaluations."""
    from fuzz_gen import rand_objects
    rng, cfg, nodes, existing, names = rand_cluster(40 + seed, n_nodes=400 + 100 * seed, n_existing=400, cfg_index=0)
    objs = rand_objects(rng)
    seq = _build(cfg, nodes, existing)
    par = _build(dict(cfg, cpuThreads=16), nodes, existing)
    for ob in objs:
        seq.upsert_object(ob)
        par.upsert_object(ob)
    try:
        for k in range(60):
            pod = rand_pod(rng, k, names)
            rs, es = seq.schedule_one(seq.compile(pod), assume=True, evaluate=True)
            rp, ep = par.schedule_one(par.compile(pod), assume=True, evaluate=True)
            assert rs.as_tuple() == rp.as_tuple(), f"pod {k}"
            for key in es:
                assert es[key] == ep[key], f"pod {k}: eval[{key}]"
    finally:
        seq.close()
        par.close()

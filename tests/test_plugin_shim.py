"""The plugin-level drop-in (INTEGRATION.md `Shim`) under the framework's own loop.

kube-scheduler's framework, replayed step by step (`shim_replay.Framework`: RunPreFilterPlugins, the
rotated Filter loop with the first failure winning, RunPreScorePlugins' Skip, RunScorePlugins' Score /
NormalizeScore / [0, 100] check / profile weights, heap selectHost), drives one Shim instance per plugin
over ONE evaluation of the library (`ksg_schedule_one` without assume, `ksg_eval_out`).  Its
ScheduleResult must equal the reference algorithm's (the oracle's own cycle, with assume) pod by pod,
and the framework's AssumePod reaches the library as the cache event it is (`ksg_add_pod`).

The CPU test drives the shim over liboracle.so (the same ABI); the gpu test over libksg.so.
"""
import copy

import pytest

from fuzz_gen import namespaces, rand_cluster, rand_pod
from oracle_binding import oracle
from shim_replay import Framework

SUCCESS = 0


def _feed(b, nodes, existing):
    for ns in namespaces():
        b.upsert_namespace(ns)
    for n in nodes:
        b.add_node(n)
    for p in existing:
        b.add_pod(p)


def run_shim_stream(make_lib, seed, n_nodes, n_existing, n_pods, cfg_index=None):
    rng, cfg, nodes, existing, names = rand_cluster(seed, n_nodes=n_nodes, n_existing=n_existing, cfg_index=cfg_index)
    lib, ref = make_lib(cfg), oracle(cfg)
    _feed(lib, nodes, existing)
    _feed(ref, nodes, existing)
    n = lib.num_nodes()
    assert lib.node_names() == ref.node_names()
    fw = Framework(cfg)
    placed = 0
    for k in range(n_pods):
        pod = rand_pod(rng, k, names)
        tag = f"seed {seed} pod {k}"
        h = lib.compile(pod)
        _, ev = lib.schedule_one(h, assume=False, evaluate=True)  # the first PreFilter of the cycle
        got = fw.schedule_pod(ev, n)
        ro, eo = ref.schedule_one(ref.compile(pod), assume=True, evaluate=True)
        assert got == ro.as_tuple(), f"{tag}: framework over the shim {got} != reference {ro.as_tuple()}"
        for key in ("plugin_scores", "normalized_scores", "total_scores", "score_plugin_mask"):
            assert ev[key] == eo[key], f"{tag}: {key} differs from the reference"
        for p in range(len(ev["normalized_scores"])):
            if ev["score_plugin_mask"] >> p & 1:  # what Score hands RunScorePlugins is a valid score
                assert all(0 <= s <= 100 for s in ev["normalized_scores"][p]), f"{tag}: plugin {p} out of range"
        lib.release(h)
        if got[0] == SUCCESS:  # Scheduler.assume -> Cache.AssumePod, forwarded to the library
            bound = copy.deepcopy(pod)
            bound["spec"]["nodeName"] = lib.node_names()[got[1]]
            lib.add_pod(bound)
            placed += 1
    return placed


@pytest.mark.parametrize("seed", range(8))
def test_shim_over_oracle_abi_matches_reference(seed):
    """CPU: the shim over liboracle.so's identical ABI (no device)."""
    placed = run_shim_stream(oracle, 7100 + seed, n_nodes=[9, 60, 130, 257][seed % 4], n_existing=40, n_pods=30,
                             cfg_index=seed % 8)
    assert placed > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(16))
def test_shim_over_device_matches_reference(seed):
    """GPU: the shim over libksg.so -- every plugin's Score in [0, 100], the framework's weighted sum
    and heap pop reproduce the reference's TotalScores and chosen node."""
    from ksg.native import Scheduler
    placed = run_shim_stream(Scheduler, 7200 + seed, n_nodes=[9, 60, 130, 257, 300, 600][seed % 6], n_existing=60,
                             n_pods=40, cfg_index=seed % 8)
    assert placed > 0

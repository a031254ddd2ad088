"""OpportunisticBatching in the oracle (CPU): the state machine against the reference's own TestBatchBasic
vectors (tests/golden/batch_basic.json, make_fixtures_j.py), and the restatement wired into schedulePod on
scheduler_perf's batching workloads (test/integration/scheduler_perf/batching/performance-config.yaml)."""
import ctypes as C
import json
import os

import pytest

from oracle_binding import load, oracle

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "batch_basic.json")))["cases"]

# scheduler-config-no-topology.yaml: PodTopologySpread with List defaulting and no default constraints
NO_TOPOLOGY = {"podTopologySpread": {"defaultingType": "List", "defaultConstraints": []}}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_batch_basic_vectors(case):
    lib = load()
    lib.ksgo_debug_batch_basic.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
    b = json.dumps(case).encode()
    out = C.create_string_buffer(4096)
    assert lib.ksgo_debug_batch_basic(b, len(b), out, 4096) == 0, out.value
    got = json.loads(out.value.decode())
    assert got["hint"] == case["expectedHint"]
    want = case["expectedState"]
    assert got["empty"] == (want is None)
    if want is not None:
        assert got["signature"] == want["signature"] and got["sortedNodes"] == want["sortedNodes"]


def _hinted(r):  # a hinted placement: the hinted node alone was evaluated (schedulePod's one-node path)
    return r.status == 0 and r.evaluated_nodes == 1 and r.feasible_nodes == 1


@pytest.mark.parametrize("workload", ["hostport", "saturation"])
def test_batching_workloads_take_hints(workload):
    """HostPortConflict / ResourceSaturation (one pod per node): after the first full cycle every pod is
    placed on the next node of the stored heap, without a full pass; with the gate off, every pod runs a
    full cycle; on these one-pod-per-node streams both place every pod."""
    from ksg.synth import batching
    nodes, pods = batching(60, 60, workload)
    res = {}
    for gate in (True, False):
        o = oracle(dict(NO_TOPOLOGY, featureGates={"OpportunisticBatching": gate}))
        for n in nodes:
            o.add_node(n)
        res[gate] = [o.schedule_one(o.compile(p), assume=True)[0] for p in pods]
    hints = sum(_hinted(r) for r in res[True][1:])
    assert hints >= 55, hints
    assert not any(_hinted(r) for r in res[False])
    assert all(r.status == 0 for r in res[True]) and all(r.status == 0 for r in res[False])
    assert len({r.node_index for r in res[True]}) == 60


def test_default_profile_is_inert():
    """Under the default profile PodTopologySpread refuses to sign every pod (plugin.go:92-102): no hints."""
    from ksg.synth import batching
    nodes, pods = batching(40, 40, "hostport")
    o = oracle({})
    for n in nodes:
        o.add_node(n)
    rs = [o.schedule_one(o.compile(p), assume=True)[0] for p in pods]
    assert not any(_hinted(r) for r in rs)


def test_expiry_and_clock():
    """maxBatchAge (batch.go:57): a pod more than 500 ms after the state was stored gets no hint."""
    from ksg.synth import batching
    nodes, pods = batching(30, 30, "hostport")
    o = oracle(NO_TOPOLOGY)
    lib = load()
    lib.ksgo_set_clock.argtypes = [C.c_void_p, C.c_int64]
    for n in nodes:
        o.add_node(n)
    t = 10 ** 12
    out = []
    for k, p in enumerate(pods[:6]):
        t += 600 * 10 ** 6 if k == 3 else 10 ** 6  # pod 3 comes 600 ms later
        lib.ksgo_set_clock(C.c_void_p(o.ctx), t)
        out.append(_hinted(o.schedule_one(o.compile(p), assume=True)[0]))
    assert out == [False, True, True, False, True, True]


def test_clock_step_expires_state_inside_a_batch():
    """ksgo_debug_clock_step: each cycle reads the clock (batch.go:202) and the fixed clock advances per read, so
    one schedule_batch call expires the stored state (maxBatchAge 500 ms) the way separate cycles would: with
    a 300 ms step the state a pod stores is 300 ms old at the next pod (hint), then 600 ms at the one after --
    but each hinted pod keeps the state (its creation time is that of the pod that stored it), so hints come
    only every second pod."""
    from ksg.synth import batching
    nodes, pods = batching(30, 30, "hostport")
    seq = {}
    for step in (0, 300):
        o = oracle(NO_TOPOLOGY)
        for n in nodes:
            o.add_node(n)
        o.set_clock(10 ** 12)
        o.clock_step(step * 10 ** 6)
        seq[step] = [_hinted(r) for r in o.schedule_batch([o.compile(p) for p in pods[:8]], assume=True)]
    assert seq[0] == [False] + [True] * 7
    assert seq[300] == [False, True, False, True, False, True, False, True]

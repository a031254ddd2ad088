"""The node-sharded exchange protocol, world_size 2 over torch.distributed gloo.

This is the CPU rehearsal of what k_xpack_a / k_select_shard / k_commit do around the RCCL
all-reduces: every rank owns a contiguous range of the snapshot order, publishes its feasible
count (and the count before nextStartNodeIndex) in its own slot of a MAX-reduced vector, derives
global feasible positions from the reduced slots, packs (TotalScore, heap pre-order key) for its
nodes, and publishes its best (key, node); the winner is the max key over the ranks.  Also the
percentageOfNodesToScore cut (k_sample_shard_a/b, (c) below).  Checked
against (a) the oracle's container/heap root (ksgo_heap_root) on tie-heavy score lists with
random rotations, and (b) the oracle's chosen node over a scheduling stream, whose TotalScores
the oracle computes with the unsharded NormalizeScore maxima.  The word layout, the (TotalScore,
pre-order) key and the persistent loops' exchange-A granule packing come from libksg.so
(ksg_debug_exchange_layout / _pack_best / _gran_a: desc.h itself, no Python copy); (d) the
persistent loop's granule exchange of counts and maxima over participants; (e) the
PodTopologySpread histogram protocol -- each rank's partial zone counts and domain presence over
its node shard, merged (sum / max) as k_agg_loop merges its shared-region partials, the DoNotSchedule
minimum over present domains, and every rank's filter verdicts against the oracle's.
"""
import ctypes as C
import os
import random

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAYOUT_NAMES = ["kMaxShards", "XA_CNT", "XA_BELOW", "XA_NONIGN", "XA_MAX_TAINT", "XA_MAX_NA", "XA_MAX_IPA",
                "XA_NMIN_IPA", "XA_END", "XA_PROC", "XA_WORDS", "XB_KEY", "XB_NODE", "XB_WORDS", "XP_MAX_PTS",
                "XP_NMIN_PTS", "XP_WORDS", "XS_CNT", "XS_BELOW", "XS_WORDS", "kPreBits"]


def ksg_lib():
    """libksg.so's host-side layout exports (desc.h); no device is touched."""
    lib = C.CDLL(os.path.join(ROOT, "kubernetes-kubernetes_amd", "lib", "libksg.so"))
    lib.ksg_debug_exchange_layout.argtypes = [C.POINTER(C.c_int32), C.c_int32]
    lib.ksg_debug_pack_best.restype = C.c_uint64
    lib.ksg_debug_pack_best.argtypes = [C.c_int64, C.c_uint32]
    lib.ksg_debug_gran_a.restype = C.c_uint64
    lib.ksg_debug_gran_a.argtypes = [C.c_int32, C.c_uint32, C.c_uint32, C.c_int64, C.c_int64]
    lib.ksg_debug_gran_a_decode.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                            C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    return lib


def layout(lib):
    buf = (C.c_int32 * 64)()
    n = lib.ksg_debug_exchange_layout(buf, 64)
    assert n == len(LAYOUT_NAMES)
    return dict(zip(LAYOUT_NAMES, buf[:n]))


LIB = None
L = None


def _init_layout():
    global LIB, L
    if LIB is None:
        LIB = ksg_lib()
        L = layout(LIB)


def pack_best(total, p):  # desc.h pack_best through the library
    return LIB.ksg_debug_pack_best(total, p)


def preorder_pos(key):  # desc.h preorder_pos (the key's low kPreBits bits hold its complement)
    ln = key & 31
    return ((key >> 5) >> (24 - ln)) - 1


def shard(n, world, rank, blk=256):
    nb = (n + blk - 1) // blk
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    return min(b0 * blk, n), min(b1 * blk, n)


def allreduce_max(vals):
    t = torch.tensor(vals, dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()


def sharded_select(feasible, totals, start, world, rank, blk):
    """-> winning snapshot index (or -1), exactly the device protocol."""
    n = len(feasible)
    lo, hi = shard(n, world, rank, blk)
    mine = [i for i in range(lo, hi) if feasible[i]]
    xa = [0] * L["XA_WORDS"]
    xa[L["XA_CNT"] + rank] = len(mine)
    xa[L["XA_BELOW"] + rank] = sum(1 for i in mine if i < start)
    xa = allreduce_max(xa)
    F = sum(xa[L["XA_CNT"]:L["XA_CNT"] + world])
    pre = sum(xa[L["XA_CNT"]:L["XA_CNT"] + rank])
    before = sum(xa[L["XA_BELOW"]:L["XA_BELOW"] + world])
    best, node = 0, -1
    for j, i in enumerate(mine):
        g = pre + j
        pos = g - before if g >= before else g + F - before
        k = pack_best(totals[i], pos)
        if k > best:
            best, node = k, i
    xb = [0] * L["XB_WORDS"]
    xb[L["XB_KEY"] + rank] = best
    xb[L["XB_NODE"] + rank] = node + 1 if node >= 0 else 0
    xb = allreduce_max(xb)
    w = max(range(world), key=lambda r: xb[L["XB_KEY"] + r])
    if F == 0:
        return -1
    # every rank must be able to recover the winner's node from its slot
    assert xb[L["XB_NODE"] + w] > 0
    return xb[L["XB_NODE"] + w] - 1


def sharded_cut(feasible, start, K, world, rank, blk):
    """-> (this rank's kept nodes, processedNodes): k_sample_shard_a/b's protocol.  XS slots carry
    every rank's feasible count and its count before the rotation start; the kept global feasible
    ranks [below, below + K) mod F become at most two node intervals of this rank; the rank holding
    the (K+1)-th feasible node publishes processedNodes + 1 (XA_PROC, MAX-reduced)."""
    n = len(feasible)
    lo, hi = shard(n, world, rank, blk)
    mine = [i for i in range(lo, hi) if feasible[i]]
    xs = [0] * L["XS_WORDS"]
    xs[L["XS_CNT"] + rank] = len(mine)
    xs[L["XS_BELOW"] + rank] = sum(1 for i in mine if i < start)
    xs = allreduce_max(xs)
    F = sum(xs[L["XS_CNT"]:L["XS_CNT"] + world])
    below = sum(xs[L["XS_BELOW"]:L["XS_BELOW"] + world])
    P = sum(xs[L["XS_CNT"]:L["XS_CNT"] + rank])
    c = len(mine)
    proc_word = 0
    if F <= K:
        kept = set(mine)
    else:
        gE = (below + K) % F
        if P <= gE < P + c:
            end = mine[gE - P]
            proc_word = (end - start + n) % n + 1
        kept = set()
        for a, e in ((below, min(below + K, F)), (0, max(0, below + K - F))):
            a, e = max(a, P), min(e, P + c)
            if a < e:
                i0, i1 = mine[a - P], mine[e - 1 - P] + 1
                kept |= {i for i in mine if i0 <= i < i1}
    proc_word = allreduce_max([proc_word])[0]
    processed = proc_word - 1 if proc_word else n
    return kept, processed


def granule_exchange(rng, world, rank, per_rank=3):
    """(d) the persistent loop's exchange A over world * per_rank participants: each packs its feasible count,
    its count before nextStartNodeIndex and its raw TaintToleration / NodeAffinity maxima with the library's
    packers (desc.h gran_a_counts / gran_a_maxima); the granules are all-gathered (every participant's store
    into every rank's array), decoded with the library and merged as the selection wave merges them."""
    for case in range(100):
        parts = []
        for _ in range(world * per_rank):  # the same draws on every rank
            c = rng.choice([0, rng.randint(1, 5000)])
            parts.append((c, rng.randint(0, c), rng.randint(0, (1 << 24) - 2), rng.randint(0, (1 << 24) - 2)))
        mine = parts[rank * per_rank:(rank + 1) * per_rank]
        words = []
        for c, bl, mt, mn in mine:
            words += [LIB.ksg_debug_gran_a(0, c, bl, mt, mn), LIB.ksg_debug_gran_a(1, c, bl, mt, mn)]
        t = torch.tensor(words, dtype=torch.int64)  # payloads < 2^48
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        F = below = 0
        tp1 = np1 = 0
        for w in out:
            for k in range(per_rank):
                cnt, bl, a, b = C.c_uint32(), C.c_uint32(), C.c_int64(), C.c_int64()
                assert LIB.ksg_debug_gran_a_decode(int(w[2 * k]), int(w[2 * k + 1]), C.byref(cnt), C.byref(bl),
                                                   C.byref(a), C.byref(b)) == 0
                F += cnt.value
                below += bl.value
                tp1, np1 = max(tp1, a.value), max(np1, b.value)
        live = [p for p in parts if p[0] > 0]
        assert F == sum(p[0] for p in parts) and below == sum(p[1] for p in parts), case
        assert tp1 == (max(p[2] for p in live) + 1 if live else 0), case
        assert np1 == (max(p[3] for p in live) + 1 if live else 0), case


def histogram_protocol(seed, world, rank, o_factory, blk=8):
    """(e) PodTopologySpread DoNotSchedule counts across node shards (filtering.go:255-341): each rank counts the
    matching pods on its eligible nodes per zone and marks the zones present there; the partials are summed and
    the presence merged (k_agg_loop: every participant adds its shared-region partials into every rank's
    region); the minimum over present zones gives each rank's verdict for its own nodes, which must be the
    oracle's PodTopologySpread verdicts, over a stream of assumed spread pods."""
    from ksg.synth import pod_default, pod_with_topology_spreading, NodeW
    rng = random.Random(seed + 1)
    zones = ["moon-1", "moon-2", "moon-3"]
    nodes = []
    for i in range(66):
        w = NodeW(f"hn-{i:03d}").capacity({"cpu": "64", "memory": "256Gi", "pods": "110"})
        w.label("kubernetes.io/hostname", f"hn-{i:03d}")
        if i % 11 != 5:  # a few nodes lack the key: UnschedulableAndUnresolvable
            w.label("topology.kubernetes.io/zone", zones[i % 3])
        nodes.append(w.obj())
    o = o_factory({})
    for nd in nodes:
        o.add_node(nd)
    names = o.node_names()
    zone_of = {nd["metadata"]["name"]: nd["metadata"]["labels"].get("topology.kubernetes.io/zone") for nd in nodes}
    on_node = {n: 0 for n in names}  # pods matching the constraint (color=blue, namespace sched-1) per node
    skewed = [n for n in names if zone_of[n] == "moon-1"]
    for k in range(24):  # an uneven start: blue pods on moon-1, others anywhere
        p = pod_with_topology_spreading(f"seed-{k}", "sched-1")
        p["spec"].pop("topologySpreadConstraints")
        node = skewed[rng.randrange(len(skewed))]
        p["spec"]["nodeName"] = node
        o.add_pod(p)
        on_node[node] += 1
    for k in range(30):
        p = pod_default(f"other-{k}", ns="sched-1", node=names[rng.randrange(len(names))])
        o.add_pod(p)
    n = len(names)
    lo, hi = shard(n, world, rank, blk)
    seen = [0, 0]  # verdicts on this rank's nodes: pass, fail (both must occur)
    for k in range(40):
        res, ev = o.schedule_one(o.compile(pod_with_topology_spreading(f"sp-{k}", "sched-1")), assume=True,
                                 evaluate=True)
        # this rank's partials over its shard
        cnt = [0] * len(zones)
        pres = [0] * len(zones)
        for i in range(lo, hi):
            z = zone_of[names[i]]
            if z is None:
                continue
            pres[zones.index(z)] = 1
            cnt[zones.index(z)] += on_node[names[i]]
        t = torch.tensor(cnt, dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        pz = torch.tensor(pres, dtype=torch.int64)
        dist.all_reduce(pz, op=dist.ReduceOp.MAX)
        present = [zi for zi in range(len(zones)) if pz[zi]]
        mn = min(int(t[zi]) for zi in present)
        for i in range(lo, hi):
            z = zone_of[names[i]]
            want_pts_fail = ev["node_plugin"][i] == 6 and ev["node_code"][i] != 0
            got_fail = z is None or int(t[zones.index(z)]) + 1 - mn > 5  # selfMatch 1, maxSkew 5
            assert got_fail == want_pts_fail, (k, i, got_fail, ev["node_code"][i], ev["node_plugin"][i])
            seen[got_fail] += 1
        if res.node_index >= 0:
            on_node[names[res.node_index]] += 1
    assert seen[0] and seen[1], seen


def _heap_root(lib, scores):
    arr = (C.c_int64 * len(scores))(*scores)
    return lib.ksgo_heap_root(arr, len(scores))


def _worker(rank, world, port, seed, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(root, "tests"))
        sys.path.insert(0, os.path.join(root, "kubernetes-kubernetes_amd"))
        _init_layout()
        from oracle_binding import load, oracle
        from fuzz_gen import rand_cluster, rand_pod
        lib = load()
        rng = random.Random(seed)  # same stream on every rank
        # (a) tie-heavy lists, random rotation, tiny blocks so every rank owns several
        for case in range(150):
            n = rng.randint(1, 90)
            feasible = [rng.random() < 0.7 for _ in range(n)]
            totals = [rng.choice([5, 7, 7, 9]) for _ in range(n)]
            start = rng.randrange(n)
            got = sharded_select(feasible, totals, start, world, rank, blk=rng.choice([1, 4, 16]))
            order = [i for i in list(range(start, n)) + list(range(start)) if feasible[i]]
            want = order[_heap_root(lib, [totals[i] for i in order])] if order else -1
            assert got == want, (case, got, want)
        # (c) the percentageOfNodesToScore cut: the first K feasible nodes of the rotated order and
        # processedNodes = the rotated position of the (K+1)-th (schedule_one.go:809-824,686-687)
        for case in range(200):
            n = rng.randint(1, 120)
            feasible = [rng.random() < rng.choice([0.1, 0.5, 0.9]) for _ in range(n)]
            start = rng.randrange(n)
            K = rng.randint(1, n)
            blk = rng.choice([1, 4, 16])
            kept, processed = sharded_cut(feasible, start, K, world, rank, blk)
            order = [i for i in list(range(start, n)) + list(range(start))]
            want, seen, want_proc = set(), 0, n
            for pos, i in enumerate(order):
                if feasible[i]:
                    if seen == K:
                        want_proc = pos
                        break
                    want.add(i)
                    seen += 1
            lo, hi = shard(n, world, rank, blk)
            assert kept == {i for i in want if lo <= i < hi}, (case, sorted(kept), sorted(want))
            assert processed == want_proc, (case, processed, want_proc)
        # (b) a scheduling stream: the oracle's TotalScores (unsharded normalisation), sharded argmax
        r2, cfg, nodes, existing, names = rand_cluster(seed, n_nodes=700, n_existing=60)
        o = oracle(cfg)
        for nd in nodes:
            o.add_node(nd)
        for p in existing:
            o.add_pod(p)
        start = 0  # Scheduler.nextStartNodeIndex (schedule_one.go:686-687)
        for k in range(60):
            res, ev = o.schedule_one(o.compile(rand_pod(r2, k, names)), assume=True, evaluate=True)
            feasible = [c == 0 for c in ev["node_code"]]
            if ev["prefilter_code"]:
                continue
            if res.status != 1:
                got = sharded_select(feasible, ev["total_scores"], start, world, rank, blk=256)
                assert got == res.node_index, (k, got, res.node_index)
            start = (start + res.evaluated_nodes) % len(feasible)
        granule_exchange(rng, world, rank)
        histogram_protocol(seed, world, rank, o_factory=oracle)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2])
def test_sharded_argmax_protocol_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + random.Random().randint(0, 2000)
    ps = [ctx.Process(target=_worker, args=(r, world, port, 11, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(e is None for _, e in out), out


def test_preorder_key_roundtrip():
    """desc.h pack_best (through the library): the key's low kPreBits bits give back the heap position."""
    _init_layout()
    mask = (1 << L["kPreBits"]) - 1
    for p in range(0, 1 << 20, 977):
        key = pack_best(12345, p)
        assert key >> L["kPreBits"] == 12345
        assert preorder_pos(mask - (key & mask)) == p


def test_exchange_layout_exported():
    _init_layout()
    assert L["kMaxShards"] == 8 and L["XA_WORDS"] == 4 * L["kMaxShards"] and L["XB_NODE"] == L["kMaxShards"]
    assert L["XA_PROC"] < L["XA_WORDS"] and L["XS_BELOW"] == L["kMaxShards"]

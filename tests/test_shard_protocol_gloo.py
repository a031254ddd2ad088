"""The node-sharded exchange protocol, world_size 2 over torch.distributed gloo.

This is the CPU rehearsal of what k_xpack_a / k_select_shard / k_commit do around the RCCL
all-reduces: every rank owns a contiguous range of the snapshot order, publishes its feasible
count (and the count before nextStartNodeIndex) in its own slot of a MAX-reduced vector, derives
global feasible positions from the reduced slots, packs (TotalScore, heap pre-order key) for its
nodes, and publishes its best (key, node); the winner is the max key over the ranks.  Also the
percentageOfNodesToScore cut (k_sample_shard_a/b, (c) below).  Checked
against (a) the oracle's container/heap root (ksgo_heap_root) on tie-heavy score lists with
random rotations, and (b) the oracle's chosen node over a scheduling stream, whose TotalScores
the oracle computes with the unsharded NormalizeScore maxima.
"""
import ctypes as C
import os
import random

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

XA_CNT, XA_BELOW, MAXS = 0, 8, 8
PRE_BITS = 29


def preorder_key(p):  # desc.h preorder_key
    x = p + 1
    ln = x.bit_length()
    return ((x << (24 - ln)) << 5) | ln


def preorder_pos(key):
    ln = key & 31
    return ((key >> 5) >> (24 - ln)) - 1


def pack_best(total, p):
    return (total << PRE_BITS) | ((1 << PRE_BITS) - 1 - preorder_key(p))


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
    xa = [0] * (4 * MAXS)
    xa[XA_CNT + rank] = len(mine)
    xa[XA_BELOW + rank] = sum(1 for i in mine if i < start)
    xa = allreduce_max(xa)
    F = sum(xa[XA_CNT:XA_CNT + world])
    pre = sum(xa[XA_CNT:XA_CNT + rank])
    before = sum(xa[XA_BELOW:XA_BELOW + world])
    best, node = 0, -1
    for j, i in enumerate(mine):
        g = pre + j
        pos = g - before if g >= before else g + F - before
        k = pack_best(totals[i], pos)
        if k > best:
            best, node = k, i
    xb = [0] * (2 * MAXS)
    xb[rank] = best
    xb[MAXS + rank] = node + 1 if node >= 0 else 0
    xb = allreduce_max(xb)
    w = max(range(world), key=lambda r: xb[r])
    if F == 0:
        return -1
    # every rank must be able to recover the winner's node from its slot
    assert xb[MAXS + w] > 0
    return xb[MAXS + w] - 1


def sharded_cut(feasible, start, K, world, rank, blk):
    """-> (this rank's kept nodes, processedNodes): k_sample_shard_a/b's protocol.  XS slots carry
    every rank's feasible count and its count before the rotation start; the kept global feasible
    ranks [below, below + K) mod F become at most two node intervals of this rank; the rank holding
    the (K+1)-th feasible node publishes processedNodes + 1 (XA_PROC, MAX-reduced)."""
    n = len(feasible)
    lo, hi = shard(n, world, rank, blk)
    mine = [i for i in range(lo, hi) if feasible[i]]
    xs = [0] * (2 * MAXS)
    xs[rank] = len(mine)
    xs[MAXS + rank] = sum(1 for i in mine if i < start)
    xs = allreduce_max(xs)
    F = sum(xs[:world])
    below = sum(xs[MAXS:MAXS + world])
    P = sum(xs[:rank])
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
    for p in range(0, 1 << 20, 977):
        assert preorder_pos(preorder_key(p)) == p

"""Multi-rank host logic on CPU: sharding and the QPP min/max all-reduce (gloo, world 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref_port


def test_shard_range_covers_everything():
    from qppfuse.dist import shard_range
    for n in (0, 1, 7, 3452, 1_000_000):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            sizes = [e - b for b, e in parts]
            assert max(sizes) - min(sizes) <= 1


def test_shard_by_entries_balances_ragged_lists():
    from qppfuse.dist import shard_by_entries
    rng = np.random.default_rng(0)
    R, Q = 5, 1000
    lens = rng.integers(0, 2000, Q * R)
    off = np.concatenate([[0], np.cumsum(lens)])
    for w in (2, 4, 8):
        b = shard_by_entries(off, R, w)
        assert b[0] == 0 and b[-1] == Q and np.all(np.diff(b) >= 0)
        per = [off[b[i + 1] * R] - off[b[i] * R] for i in range(w)]
        assert max(per) - min(per) <= 2 * 2000 * R


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, raw, Q, R, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qppfuse.dist import allreduce_minmax, shard_range
    b, e = shard_range(Q, world, rank)
    mine = raw[b * R:e * R].reshape(e - b, R, 13)
    mm = torch.from_numpy(np.concatenate([mine.min(axis=0).ravel(),
                                          (-mine.max(axis=0)).ravel()]).copy())
    allreduce_minmax(mm)
    out[rank] = mm.numpy().copy()
    dist.destroy_process_group()


def test_sharded_qpp_normalisation_equals_global():
    """[min, -max] per shard + MIN all-reduce == the reference's global min-max."""
    rng = np.random.default_rng(1)
    Q, R, world = 37, 3, 2
    raw = rng.normal(0, 5, (Q * R, 13))
    mgr = mp.Manager()
    out = mgr.dict()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, raw, Q, R, out), nprocs=world, join=True)
    assert np.array_equal(out[0], out[1])
    mm = out[0]
    lo, hi = mm[:R * 13].reshape(R, 13), -mm[R * 13:].reshape(R, 13)
    for r in range(R):
        res = {str(q): raw[q * R + r].tolist() for q in range(Q)}
        want = ref_port.normalize_qpp(res, "minmax")
        scale = np.where(hi[r] > lo[r], hi[r] - lo[r], 1.0)
        got = (raw[r::R] - lo[r]) / scale
        for q in range(Q):
            assert got[q].tolist() == [float(v) for v in want[str(q)]]


def _gather_worker(rank, world, port, raw, Q, R, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qppfuse.dist import allgather_qpp_raw, shard_range
    b, e = shard_range(Q, world, rank)
    mine = torch.from_numpy(raw[b * R:e * R].copy())
    pres = torch.from_numpy((np.arange(b * R, e * R) % 7 != 3))
    full, fp = allgather_qpp_raw(mine, pres)
    out[rank] = (full.numpy().copy(), fp.numpy().copy())
    dist.destroy_process_group()


def test_zscore_gathers_the_whole_table():
    """zscore needs every query in order on each rank: the gathered table equals the
    unsharded one, so per-rank device statistics equal the single-GPU ones."""
    rng = np.random.default_rng(2)
    Q, R, world = 41, 3, 2
    raw = rng.normal(0, 5, (Q * R, 13))
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gather_worker, args=(world, _free_port(), raw, Q, R, out), nprocs=world, join=True)
    for rank in range(world):
        full, fp = out[rank]
        assert full.tobytes() == raw.tobytes()
        assert np.array_equal(fp, np.arange(Q * R) % 7 != 3)


def _topk_worker(rank, world, port, sizes, out, async_op=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qppfuse.dist import gather_fused_topk
    n = sizes[rank]
    docid = torch.arange(n * 2 * 3, dtype=torch.int32).reshape(n, 2, 3) + 1000 * rank
    score = docid.to(torch.float64) / 7
    if async_op:  # bench.py's pipelined form: two gathers in flight, waited in order
        p1 = gather_fused_topk(docid, score, dst=0, sizes=sizes, async_op=True)
        p2 = gather_fused_topk(docid + 1, score, dst=0, sizes=sizes, async_op=True)
        res, res2 = p1.wait(), p2.wait()
        if res2 is not None:
            assert torch.equal(res2[0], res[0] + 1)
    else:
        res = gather_fused_topk(docid, score, dst=0)
    out[rank] = None if res is None else (res[0].numpy().copy(), res[1].numpy().copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("async_op", [False, True])
def test_gather_fused_topk_concatenates_shards_in_rank_order(async_op):
    """Unequal shards (the shard_range remainder) are padded for the collective and
    trimmed: rank 0 holds every rank's rows in rank order, the others None."""
    sizes = [3, 2]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_topk_worker, args=(2, _free_port(), sizes, out, async_op), nprocs=2, join=True)
    assert out[1] is None
    d, s = out[0]
    want = np.concatenate([np.arange(n * 6, dtype=np.int32).reshape(n, 2, 3) + 1000 * r
                           for r, n in enumerate(sizes)])
    np.testing.assert_array_equal(d, want)
    assert s.tobytes() == (want.astype(np.float64) / 7).tobytes()


def _topk_gather_worker(rank, world, port, sizes, M, k, steps, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qppfuse.dist import TopkGather
    g = TopkGather(sizes, M, k, "cpu", dst=0)
    n = sizes[rank]
    ptrs = {(t.data_ptr(), u.data_ptr()) for t, u in (g.buffers(i) for i in range(2))}
    pending, got = None, []
    for step in range(steps):  # bench.py's pipelined loop: wait for the previous, then start
        if pending is not None:
            got.append(_copy(pending.wait()))
        d, s = g.buffers(step)
        assert d.shape == (n, M, k) and (d.data_ptr(), s.data_ptr()) in ptrs  # no new buffers
        d.copy_(torch.arange(n * M * k, dtype=torch.int32).reshape(n, M, k) + 100000 * rank
                + 10 * step)
        s.copy_(d.to(torch.float64) / 3)
        pending = g.start(step)
    got.append(_copy(pending.wait()))
    out[rank] = got
    dist.destroy_process_group()


def _copy(res):
    if res is None:
        return None
    return [(d.numpy().copy(), s.numpy().copy()) for d, s in res]


@pytest.mark.parametrize("world,total", [(4, 11157), (2, 10), (8, 1000)])
def test_topk_gather_preallocated_unequal_shards(world, total):
    """dist.TopkGather (bench.py's allocation-free N > 1 gather) with C4's unequal
    shard_range(11157, 4, r) shards (2790, 2789, 2789, 2789) on gloo, world 4:
    three pipelined steps through the two buffer sets, one gather per step (docids
    and scores in one byte buffer); rank 0 holds every rank's rows, in rank order,
    trimmed to each shard."""
    from qppfuse.dist import shard_range
    sizes = [e - b for b, e in (shard_range(total, world, r) for r in range(world))]
    M, k, steps = 2, 3, 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_topk_gather_worker, args=(world, _free_port(), sizes, M, k, steps, out),
             nprocs=world, join=True)
    for r in range(1, world):
        assert out[r] == [None] * steps
    for step, per in enumerate(out[0]):
        assert len(per) == world
        for r, (d, s) in enumerate(per):
            want = np.arange(sizes[r] * M * k, dtype=np.int32).reshape(sizes[r], M, k) \
                + 100000 * r + 10 * step
            np.testing.assert_array_equal(d, want)
            assert s.tobytes() == (want.astype(np.float64) / 3).tobytes()


def _topk_rows(off, R, k, methods, docid, score):
    """[Q, M, k] top-k (docid, score) rows of every query of a run set through the C
    oracle (what engine.fused_topk packs on device): rank i's docid and score, padded
    with docid -1 / NaN past the union."""
    from oracle import _loader as coracle
    Q = (len(off) - 1) // R
    d = np.full((Q, len(methods), k), -1, np.int32)
    s = np.full((Q, len(methods), k), np.nan)
    for m, name in enumerate(methods):
        ud, uc, perm, fz = coracle.fuse(off, docid, score, R, name, 60)
        for q in range(Q):
            b, n = int(off[q * R]), min(int(uc[q]), k)
            d[q, m, :n] = ud[b + perm[b:b + n].astype(np.int64)].view(np.int32)
            s[q, m, :n] = fz[b:b + n]
    return d, s


def _entries_shard_worker(rank, world, port, off, docid, score, R, k, methods, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from qppfuse.dist import TopkGather, shard_by_entries
    plan = shard_by_entries(off, R, world)  # every rank derives the same boundaries
    b, e = int(plan[rank]), int(plan[rank + 1])
    sizes = np.diff(plan).tolist()
    g = TopkGather(sizes, len(methods), k, "cpu", dst=0)
    dd, ss = g.buffers(0)
    d, s = _topk_rows(off[b * R:e * R + 1], R, k, methods, docid, score)  # this rank's shard
    dd[:e - b].copy_(torch.from_numpy(d))
    ss[:e - b].copy_(torch.from_numpy(s))
    res = g.start(0).wait()
    out[rank] = None if res is None else [(x.numpy().copy(), y.numpy().copy()) for x, y in res]
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_shard_by_entries_ragged_gather_equals_single_process(world):
    """bench.py's total-split workloads (C3, C4) shard by Σ entries (SURVEY §8(e):
    "balanced by Σ_r K_qr"), not by query count: on ragged lists (0-1,500 entries per
    list, some queries 10x heavier) each rank fuses its dist.shard_by_entries shard,
    packs its top-k rows and TopkGather collects them on rank 0 (gloo) — the gathered
    rows, concatenated in rank order, equal a single process's rows for every query,
    and the shards' entry totals are balanced to within one query."""
    rng = np.random.default_rng(11)
    R, Q, k, methods = 3, 60, 20, ["combsum", "rrf"]
    lens = rng.integers(0, 150, Q * R)
    lens[rng.integers(0, Q * R, 12)] = rng.integers(900, 1500, 12)  # heavy queries
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    docid = np.concatenate([rng.choice(5000, n, replace=False) for n in lens]).astype(np.uint32)
    score = np.concatenate([np.sort(rng.random(n))[::-1] for n in lens])
    from qppfuse.dist import shard_by_entries
    plan = shard_by_entries(off, R, world)
    per = np.array([int(off[plan[i + 1] * R] - off[plan[i] * R]) for i in range(world)])
    qtot = off[R::R] - off[:-1:R]
    # every boundary within half a query of its target: each shard within one query
    assert np.abs(per - off[-1] / world).max() <= qtot.max()
    want_d, want_s = _topk_rows(off, R, k, methods, docid, score)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_entries_shard_worker,
             args=(world, _free_port(), off, docid, score, R, k, methods, out),
             nprocs=world, join=True)
    got = out[0]
    assert len(got) == world
    d = np.concatenate([x for x, _ in got])
    s = np.concatenate([y for _, y in got])
    np.testing.assert_array_equal(d, want_d)
    assert s.tobytes() == want_s.tobytes()

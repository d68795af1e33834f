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

"""One rank of tests/test_gpu_rccl.py (started by torch.distributed.run, backend nccl =
RCCL): the path's two collectives on device buffers — the QPP [min, -max] MIN
all-reduce and the fused top-k gather (async, waited on the stream as bench.py
pipelines it) — checked against the local values.  Prints "rccl-ok" on success."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "qpp-fusion-rag_amd"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ["LOCAL_RANK"])
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl"
    world, rank = dist.get_world_size(), dist.get_rank()
    from qppfuse import engine
    from qppfuse.dist import PendingGather
    Q, R, K = 48, 5, 1000
    methods = ["combsum", "rrf", "wcombsum"]

    def shard(r):
        """Rank r's inputs, regenerable on any rank (counter-based generator, seeded text)."""
        import numpy as np
        off, docid, raw = engine.synth_runs(r * Q, Q, R, K, seed=11)
        g = np.random.default_rng([11, r])
        nt = torch.from_numpy(g.integers(1, 12, Q).astype(np.int32)).to(dev)
        tf = torch.from_numpy(g.random((Q, 2))).to(dev)
        return off, docid, raw, nt, tf

    def fuse_shard(r, mm):
        off, docid, raw, nt, tf = shard(r)
        _, micro = engine.minmax_per_query(raw, off, want_norm=False)
        qraw = engine.qpp_raw(raw, off, R, 100, nt, tf)
        w = engine.qpp_normalize(qraw, mm, off, R, "minmax", 5)["weights"]
        out = engine.fuse(off, docid, micro, R, methods, 60, weights=w, max_entries=R * K)
        return out, off

    off, docid, raw, nt, tf = shard(rank)
    qraw = engine.qpp_raw(raw, off, R, 100, nt, tf)
    mm = engine.qpp_colminmax(qraw, off, R)
    want = mm.clone()
    work = dist.all_reduce(mm, op=dist.ReduceOp.MIN, async_op=True)
    work.wait()
    assert torch.equal(mm, want) if world == 1 else bool((mm <= want).all())
    out, off = fuse_shard(rank, mm)
    d, s = engine.fused_topk(out, off, R, 100)
    dl = [torch.empty_like(d) for _ in range(world)] if rank == 0 else None
    sl = [torch.empty_like(s) for _ in range(world)] if rank == 0 else None
    works = [dist.gather(d, dl, dst=0, async_op=True), dist.gather(s, sl, dst=0, async_op=True)]
    got = PendingGather(works, dl, sl, [Q] * world).wait()
    torch.cuda.synchronize()
    if rank == 0:
        gd, gs = got
        assert gd.shape == (world * Q, 3, 100)
        assert torch.equal(gd[:Q], d) and torch.equal(gs[:Q].view(torch.int64), s.view(torch.int64))
    # bench.py's allocation-free form: fused_topk straight into the send buffer
    # (docids and scores in one byte buffer), one gather per step, two steps pipelined
    from qppfuse.dist import TopkGather
    g = TopkGather([Q] * world, 3, 100, dev)
    pending = None
    for step in range(2):
        if pending is not None:
            pending.wait()
        engine.fused_topk(out, off, R, 100, dest=g.buffers(step))
        pending = g.start(step)
    per = pending.wait()
    torch.cuda.synchronize()
    if rank == 0:
        # every rank's rows: rank 0 regenerates each shard and fuses it with the
        # global (all-reduced) QPP min / max — the rows must match byte for byte
        assert len(per) == world
        for r in range(world):
            o_r, off_r = fuse_shard(r, mm)
            d_r, s_r = engine.fused_topk(o_r, off_r, R, 100)
            pd_, ps_ = per[r]
            assert torch.equal(pd_, d_r), r
            assert torch.equal(ps_.view(torch.int64), s_r.view(torch.int64)), r
    dist.barrier()
    dist.destroy_process_group()
    print("rccl-ok", flush=True)


if __name__ == "__main__":
    main()

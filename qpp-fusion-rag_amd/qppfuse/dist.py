"""Query sharding across GPUs (one process per GPU) and the one collective of the path.

Fusion is independent per query; QPP normalisation couples the queries of each
retriever through per-column min / max (src/qpp.py:347-361).  Each rank reduces
its shard to [min, -max] per (retriever, column) (qf_qpp_colminmax) and one
element-wise MIN all-reduce (RCCL over xGMI with backend "nccl"; gloo in the CPU
tests) combines them.  zscore normalisation (numpy's mean / std, whose pairwise
sum depends on every query's position) cannot be combined from shard partials
bit-exactly: allgather_qpp_raw gives every rank the whole raw predictor table
(R*13 doubles + one presence flag per query — 0.5 MB per 1,000 queries at R = 5)
and each rank computes the statistics itself.  Fused lists stay on the rank that
produced them.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_range(n_queries: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [begin, end) of `n_queries` for `rank` of `world`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_queries, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def shard_by_entries(list_off: np.ndarray, n_retrievers: int, world: int) -> np.ndarray:
    """Query boundaries [world+1] balancing Σ entries (ragged lists) across ranks
    (shards balanced by Σ_r K_qr): boundary r is the query boundary
    nearest to r/world of the entries, so each lies within half a query of its
    target.  Contiguous query ranges, in query order."""
    qoff = np.asarray(list_off, dtype=np.int64)[:: n_retrievers]
    qoff = qoff - qoff[0]  # (a slice of a larger run set: offsets relative to its start)
    total = int(qoff[-1])
    targets = np.array([total * r // world for r in range(world + 1)], dtype=np.int64)
    hi = np.clip(np.searchsorted(qoff, targets, side="left"), 0, len(qoff) - 1)
    lo = np.clip(hi - 1, 0, len(qoff) - 1)
    b = np.where(targets - qoff[lo] < qoff[hi] - targets, lo, hi)
    b[0], b[-1] = 0, len(qoff) - 1
    return np.maximum.accumulate(b)


def allreduce_minmax(mm, group=None, async_op=False):
    """In-place element-wise MIN over ranks of the [min, -max] buffer (a torch tensor).
    async_op=True returns the work handle (None on one rank): launch independent
    kernels, then handle.wait() before reading mm — the exchange hides behind them."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        work = dist.all_reduce(mm, op=dist.ReduceOp.MIN, group=group, async_op=async_op)
        return work if async_op else mm
    return None if async_op else mm


def allgather_qpp_raw(raw, present, group=None):
    """All ranks' raw predictor rows [q*R + r, 13] and presence flags [q*R + r]
    (contiguous query shards, in rank order) concatenated on every rank."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return raw, present
    world = dist.get_world_size(group)
    n = torch.tensor([raw.shape[0]], dtype=torch.int64, device=raw.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    m = max(sizes)
    pad = torch.zeros((m, raw.shape[1]), dtype=raw.dtype, device=raw.device)
    pad[: raw.shape[0]] = raw
    ppad = torch.zeros(m, dtype=torch.int64, device=raw.device)
    ppad[: raw.shape[0]] = present.to(torch.int64)
    rows = [torch.empty_like(pad) for _ in range(world)]
    pres = [torch.empty_like(ppad) for _ in range(world)]
    dist.all_gather(rows, pad, group=group)
    dist.all_gather(pres, ppad, group=group)
    return (torch.cat([t[:k] for t, k in zip(rows, sizes)]),
            torch.cat([t[:k] for t, k in zip(pres, sizes)]).to(torch.bool))


class PendingGather:
    """An in-flight gather_fused_topk(async_op=True): wait() makes the caller's
    stream wait for the collective (no host block on RCCL) and returns the
    concatenated (docid, score) on the destination rank, None elsewhere."""

    def __init__(self, works, dl, sl, sizes):
        self._works, self._dl, self._sl, self._sizes = works, dl, sl, sizes

    def wait(self):
        import torch
        for w in self._works:
            w.wait()
        if self._dl is None:
            return None
        k = self._sizes
        return (torch.cat([t[:n] for t, n in zip(self._dl, k)]),
                torch.cat([t[:n] for t, n in zip(self._sl, k)]))


def gather_fused_topk(docid, score, dst: int = 0, group=None, sizes=None, async_op=False):
    """The final fused top-k of every rank's query shard, concatenated in rank
    order on rank `dst` (None elsewhere): docid [Q_r, M, k] and score tensors
    from engine.fused_topk.  Shards may differ in size by the shard_range
    remainder: rows are padded to the largest shard for the collective
    (dist.gather over RCCL/xGMI; gloo in the CPU tests) and trimmed after.
    `sizes` (every rank's row count, when the caller knows them — fixed shards)
    skips the all-gather of the counts and its host synchronisation.
    async_op=True returns a PendingGather at once (the collective runs on the
    communicator's stream beside whatever the caller launches next)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return PendingGather([], [docid], [score], [docid.shape[0]]) if async_op else (docid, score)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if dist.get_backend(group) == "gloo" and docid.is_cuda:  # gloo rehearsal: host buffers
        docid, score = docid.cpu(), score.cpu()
    if sizes is None:
        n = torch.tensor([docid.shape[0]], dtype=torch.int64, device=docid.device)
        got = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(got, n, group=group)
        sizes = [int(s.item()) for s in got]
    sizes = list(sizes)
    if len(sizes) != world or sizes[rank] != docid.shape[0]:
        raise ValueError(f"sizes {sizes} do not match this rank's {docid.shape[0]} rows")
    m = max(sizes)
    pad = lambda t, v: torch.cat([t, t.new_full((m - t.shape[0],) + tuple(t.shape[1:]), v)]) \
        if t.shape[0] < m else t
    d, s = pad(docid, -1), pad(score, float("nan"))
    dl = [torch.empty_like(d) for _ in range(world)] if rank == dst else None
    sl = [torch.empty_like(s) for _ in range(world)] if rank == dst else None
    works = [dist.gather(d, dl, dst=dst, group=group, async_op=async_op),
             dist.gather(s, sl, dst=dst, group=group, async_op=async_op)]
    pending = PendingGather([w for w in works if w is not None] if async_op else [],
                            dl if rank == dst else None, sl, sizes)
    return pending if async_op else pending.wait()


class TopkGather:
    """The per-step top-k gather of fixed shards, allocation-free (bench.py's timed
    N > 1 step): every buffer is made once.

    * `depth` sets of send buffers [m, M, k] (m = the largest shard), padding rows
      pre-filled with docid -1 / NaN; engine.fused_topk writes this rank's rows
      straight into the first sizes[rank] rows (`buffers(i)`), so nothing is
      padded or copied per step;
    * on `dst`, `depth` receive buffers [world, bytes], one contiguous block per
      set; dist.gather lands every rank's buffer in a row of it (the views are made
      once).  result(i) returns per-rank (docid, score) views trimmed to each shard.
    With the gloo backend and device tensors (the one-GPU rehearsal) the send and
    receive sides go through preallocated host buffers.
    A rank's docids and scores share one byte buffer (docids first, the scores at
    the next 8-byte boundary), so a step is ONE gather (RCCL: one set of
    point-to-point sends into dst) instead of one per column.
    Step i uses set i % depth: with depth 2 and the pipelined wait (step i waits for
    step i-1's gather before queuing step i+1), a set is never rewritten in flight.
    Bytes per step into dst: world * m * M * k * (4 + 8).
    """

    def __init__(self, sizes, M: int, k: int, device, dst: int = 0, group=None, depth: int = 2):
        import torch
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        self.sizes = [int(x) for x in sizes]
        if len(self.sizes) != self.world:
            raise ValueError(f"{len(self.sizes)} shard sizes for {self.world} ranks")
        self.M, self.k, self.dst, self.group, self.depth = int(M), int(k), dst, group, depth
        self.m = max(self.sizes)
        dev = torch.device(device)
        self.host = dist.get_backend(group) == "gloo" and dev.type == "cuda"
        cells = self.m * self.M * self.k
        self._soff = (4 * cells + 7) // 8 * 8  # the scores' byte offset
        self.nbytes = self._soff + 8 * cells
        self.send = [torch.empty(self.nbytes, dtype=torch.uint8, device=dev) for _ in range(depth)]
        for buf in self.send:  # padding rows: docid -1, score NaN (written once)
            d, s = self._views(buf)
            d.fill_(-1)
            s.fill_(float("nan"))
        cdev = torch.device("cpu") if self.host else dev
        if self.host:
            self.hsend = [torch.empty(self.nbytes, dtype=torch.uint8).pin_memory()
                          for _ in range(depth)]
        self.recv = None
        if self.rank == dst:
            self.recv = [torch.empty((self.world, self.nbytes), dtype=torch.uint8, device=cdev)
                         for _ in range(depth)]
            self._rl = [[row.view(torch.float64) for row in t.unbind(0)] for t in self.recv]
            self._rv = [[self._views(t[r]) for r in range(self.world)] for t in self.recv]
        n = self.sizes[self.rank]
        self._out = [tuple(v[:n] for v in self._views(buf)) for buf in self.send]

    def _views(self, buf):
        """(docid int32 [m, M, k], score float64 [m, M, k]) views of one byte buffer."""
        import torch
        shape, cells = (self.m, self.M, self.k), self.m * self.M * self.k
        return (buf[:4 * cells].view(torch.int32).view(shape),
                buf[self._soff:self._soff + 8 * cells].view(torch.float64).view(shape))

    def buffers(self, i: int):
        """(docid, score) [sizes[rank], M, k] views of set i % depth: engine.fused_topk's out."""
        return self._out[i % self.depth]

    def start(self, i: int):
        """Gather set i % depth to dst, asynchronously; returns a handle whose wait()
        makes the caller's stream wait for it (no host block on RCCL)."""
        import torch
        import torch.distributed as dist
        j = i % self.depth
        buf = self.send[j]
        mine = self.rank == self.dst
        if self.host:
            # gloo rehearsal: host buffers (the copy synchronises the stream), and the
            # two columns as two typed gathers, which gloo runs side by side (one
            # byte-buffer gather measured twice as slow there)
            self.hsend[j].copy_(buf)
            d, s = self._views(self.hsend[j])
            rv = self._rv[j] if mine else None
            works = [dist.gather(d, [x for x, _ in rv] if mine else None, dst=self.dst,
                                 group=self.group, async_op=True),
                     dist.gather(s, [y for _, y in rv] if mine else None, dst=self.dst,
                                 group=self.group, async_op=True)]
            return _TopkHandle(self, j, [w for w in works if w is not None])
        # RCCL: one gather of the whole buffer, as float64 words (a bit copy: the
        # docids pass through unchanged)
        w = dist.gather(buf.view(torch.float64), self._rl[j] if mine else None, dst=self.dst,
                        group=self.group, async_op=True)
        return _TopkHandle(self, j, [w] if w is not None else [])

    def result(self, i: int):
        """On dst: per-rank (docid, score) views trimmed to each shard (None elsewhere)."""
        if self.recv is None:
            return None
        j = i % self.depth
        return [(d[:n], s[:n]) for (d, s), n in zip(self._rv[j], self.sizes)]


class _TopkHandle:
    def __init__(self, g: TopkGather, j: int, works):
        self._g, self._j, self._works = g, j, works

    def wait(self):
        for w in self._works:
            w.wait()
        return self._g.result(self._j)

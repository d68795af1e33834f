"""Device-level entry points: torch tensors (HBM buffers) in, torch tensors out.

PyTorch is only the allocator / stream owner here; all compute is the HIP code
in libqppfuse.so, launched on torch's current stream so that RCCL collectives
(torch.distributed, backend "nccl") order correctly with the kernels.
Every function raises if no ROCm device or no library is present — there is no
CPU path.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch

from . import _lib

_MNAMES = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf", "learned", "probfuse",
           "wrrf_mul"]


def require_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("qppfuse needs a ROCm GPU (gfx950 / MI355X); it has no CPU fallback")
    _lib.lib()
    return torch.device("cuda", torch.cuda.current_device())


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("qppfuse expects contiguous device tensors")
    return t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def methods_mask(methods) -> int:
    if isinstance(methods, int):
        return methods
    mask = 0
    for m in methods:
        mask |= _lib.METHOD_BITS[m]
    return mask


def method_names(mask: int):
    return [n for i, n in enumerate(_MNAMES) if (mask >> i) & 1]


@dataclass
class FuseOut:
    """Device outputs of qf_fuse for one launch shape.  Per query, at its first
    entry's offset b: union_docid[b + u] and fused[m, b + u] in first-seen order
    (u < union_count), and perm[m, b + i] = the u of rank i — a ranked list is
    fused[m, b + perm[m, b + i]] (include/qppfuse.h)."""
    union_docid: torch.Tensor  # int32 view of uint32 [E]
    union_count: torch.Tensor  # int32 [Q]
    perm: torch.Tensor         # int16 view of uint16 [M, E] (int32 view of uint32: wide)
    fused: torch.Tensor        # float64 [M, E]
    methods: list
    list_off: Optional[torch.Tensor] = None  # the last launch's run set (ranked_fused)
    n_retrievers: int = 0

    @property
    def wide(self) -> bool:
        """uint32 perm (qf_fuse_wide: unions above 65,535 documents)."""
        return self.perm.dtype == torch.int32

    def ranked_fused(self) -> torch.Tensor:
        """[M, E] scores in rank order (rank i of a query at b + i; entries past its
        union are 0): fused gathered through perm on the device."""
        R, off = self.n_retrievers, self.list_off
        Q = (off.numel() - 1) // R
        E = self.fused.shape[1]
        qoff = off[::R][:Q + 1].to(torch.int64)
        n_q = qoff[1:] - qoff[:-1]
        q_of_e = torch.repeat_interleave(torch.arange(Q, device=off.device), n_q)
        pos = torch.arange(int(qoff[-1]), device=off.device) - qoff[:-1][q_of_e]
        ok = pos < self.union_count[:Q].to(torch.int64)[q_of_e]
        base = qoff[:-1][q_of_e]
        out = torch.zeros_like(self.fused)
        n = int(qoff[-1])
        for m in range(self.fused.shape[0]):
            u = self.perm[m, :n].to(torch.int64) & (0xFFFFFFFF if self.wide else 0xFFFF)
            idx = torch.where(ok, base + u, torch.zeros_like(u))
            out[m, :n] = torch.where(ok, self.fused[m].gather(0, idx),
                                     torch.zeros((), dtype=torch.float64, device=off.device))
        return out[:, :E]


def needs_wide(max_entries: int) -> bool:
    """Whether a query of max_entries entries needs the uint32 perm (qf_fuse_wide)."""
    return int(max_entries) > _lib.max_entries_per_query()


def alloc_fuse_out(n_queries: int, n_entries: int, mask: int, device, wide: bool = False) -> FuseOut:
    M = bin(mask).count("1")
    E = max(int(n_entries), 1)
    return FuseOut(torch.empty(E, dtype=torch.int32, device=device),
                   torch.empty(max(n_queries, 1), dtype=torch.int32, device=device),
                   torch.empty((M, E), dtype=torch.int32 if wide else torch.int16, device=device),
                   torch.empty((M, E), dtype=torch.float64, device=device),
                   method_names(mask))


def fuse(list_off: torch.Tensor, docid: torch.Tensor, score: torch.Tensor, n_retrievers: int,
         methods, rrf_k: int = 60, weights: Optional[torch.Tensor] = None,
         rank: Optional[torch.Tensor] = None, max_entries: Optional[int] = None,
         out: Optional[FuseOut] = None, seg_prob: Optional[torch.Tensor] = None,
         n_segments: int = 0, seg_len: int = 0,
         learned_f32: Optional[int] = None,
         workspace: Optional[torch.Tensor] = None, qpp=None,
         qpp_micro_out: Optional[torch.Tensor] = None) -> FuseOut:
    """qf_fuse over every query of a packed run set (see include/qppfuse.h); with
    "probfuse" among the methods, qf_fuse_probfuse with the [R, x] segment table;
    methods == ["learned"] with learned_f32 (run bitmask: float32 model weights,
    FusionMLP), qf_fuse_learned_f32.  A query above qf_max_entries_per_query()
    (65,535) entries takes the _wide entry points (uint32 perm): `out` is then
    allocated wide (alloc_fuse_out(..., wide=True)).  `workspace`: a caller-owned
    device byte buffer for the workspace kernel (qf_fuse_ws; workspace_bytes() sizes
    it) instead of the library's stream-ordered allocation.  `qpp` = (raw, stats,
    mode, qpp_index): the W-* weights from the raw QPP predictors and their column
    statistics, computed inside the fusion (qf_fuse_qpp — the weights qpp_normalize
    would give, one launch fewer); for the uint16-perm path without a workspace
    (other calls normalise first and pass `weights`).  `qpp_micro_out` (with `qpp`):
    int64 [Q * R * 13] receiving the .qpp "%.6f" micro-units of all 13 columns
    (qf_fuse_qpp_micro — qpp_normalize's "micro", written by the join)."""
    dev = require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    E = docid.numel()
    mask = methods_mask(methods)
    if score.dtype == torch.int32:
        kind = _lib.SCORE_MICRO
    elif score.dtype == torch.float64:
        kind = _lib.SCORE_F64
    else:
        raise TypeError("score must be float64 or int32 micro-units")
    if max_entries is None:
        raise ValueError("max_entries (largest per-query entry count) is required")
    wide = needs_wide(max_entries)
    if out is None:
        out = alloc_fuse_out(Q, E, mask, dev, wide=wide)
    elif wide and not out.wide:
        raise ValueError(f"max_entries {max_entries} needs a uint32 perm: "
                         "alloc_fuse_out(..., wide=True)")
    wide = out.wide
    sfx = "_wide" if wide else ""
    out.list_off, out.n_retrievers = list_off, R
    if mask & _lib.PROBFUSE:
        if seg_prob is None or seg_prob.dtype != torch.float64 or seg_prob.numel() != R * n_segments:
            raise ValueError("probfuse needs seg_prob: float64 [n_retrievers * n_segments]")
        _lib.call("qf_fuse_probfuse" + sfx, Q, R, _ptr(list_off), _ptr(docid), _ptr(score), kind,
                  _ptr(rank), _ptr(weights), mask, int(rrf_k), _ptr(seg_prob), int(n_segments),
                  int(seg_len), int(max_entries), _ptr(out.union_docid), _ptr(out.union_count),
                  _ptr(out.perm), _ptr(out.fused), out.fused.shape[1], _stream())
        return out
    if learned_f32 is not None:
        if mask != _lib.LEARNED:
            raise ValueError("learned_f32 applies to methods == ['learned'] only")
        if int(learned_f32) >> R:
            raise ValueError(f"learned_f32 names runs beyond the {R} of the run set")
        _lib.call("qf_fuse_learned_f32" + sfx, Q, R, _ptr(list_off), _ptr(docid), _ptr(score), kind,
                  _ptr(weights), int(learned_f32) & 0xFFFFFFFF, int(max_entries),
                  _ptr(out.union_docid), _ptr(out.union_count), _ptr(out.perm), _ptr(out.fused),
                  out.fused.shape[1], _stream())
        return out
    if qpp_micro_out is not None and qpp is None:
        raise ValueError("qpp_micro_out needs qpp=(raw, stats, mode, qpp_index)")
    if qpp is not None:
        raw_qpp, stats, mode, qidx = qpp
        mode_id = {"none": _lib.NORM_NONE, "minmax": _lib.NORM_MINMAX,
                   "zscore": _lib.NORM_ZSCORE}[mode]
        if wide or workspace is not None or weights is not None or mask & _lib.LEARNED:
            raise ValueError("qpp weights: the uint16-perm fusion without weights / workspace "
                             "/ learned fusion")
        if raw_qpp.dtype != torch.float64 or raw_qpp.numel() != Q * R * _lib.QPP_COLS:
            raise ValueError(f"qpp raw must be float64 [{Q * R}, {_lib.QPP_COLS}]")
        if qpp_micro_out is not None:
            if qpp_micro_out.dtype != torch.int64 or qpp_micro_out.numel() != Q * R * _lib.QPP_COLS \
                    or not qpp_micro_out.is_contiguous():
                raise ValueError(f"qpp_micro_out must be contiguous int64 [{Q * R * _lib.QPP_COLS}]")
            _lib.call("qf_fuse_qpp_micro", Q, R, _ptr(list_off), _ptr(docid), _ptr(score), kind,
                      _ptr(rank), _ptr(raw_qpp), _ptr(stats), mode_id, int(qidx), mask,
                      int(rrf_k), int(max_entries), _ptr(out.union_docid), _ptr(out.union_count),
                      _ptr(out.perm), _ptr(out.fused), out.fused.shape[1], _ptr(qpp_micro_out),
                      _stream())
            return out
        _lib.call("qf_fuse_qpp", Q, R, _ptr(list_off), _ptr(docid), _ptr(score), kind,
                  _ptr(rank), _ptr(raw_qpp), _ptr(stats), mode_id, int(qidx), mask, int(rrf_k),
                  int(max_entries), _ptr(out.union_docid), _ptr(out.union_count),
                  _ptr(out.perm), _ptr(out.fused), out.fused.shape[1], _stream())
        return out
    if workspace is not None:
        if workspace.device != out.fused.device or not workspace.is_contiguous():
            raise ValueError("workspace must be a contiguous buffer on the fusion's device")
        if workspace.data_ptr() % 256:
            raise ValueError("workspace must be 256-byte aligned (a slice such as ws[1:] is "
                             "not): its workgroup shares hold atomicCAS targets")
        _lib.call("qf_fuse_ws", Q, R, _ptr(list_off), _ptr(docid), _ptr(score), kind, _ptr(rank),
                  _ptr(weights), mask, int(rrf_k), int(max_entries), _ptr(out.union_docid),
                  _ptr(out.union_count), _ptr(out.perm), 1 if wide else 0, _ptr(out.fused),
                  out.fused.shape[1], _ptr(workspace),
                  workspace.numel() * workspace.element_size(), _stream())
        return out
    _lib.call("qf_fuse" + sfx, Q, R, _ptr(list_off), _ptr(docid), _ptr(score), kind, _ptr(rank),
              _ptr(weights), mask, int(rrf_k), int(max_entries), _ptr(out.union_docid),
              _ptr(out.union_count), _ptr(out.perm), _ptr(out.fused), out.fused.shape[1],
              _stream())
    return out


def workspace_bytes(n_queries: int, n_retrievers: int, max_entries: int, methods) -> int:
    """qf_fuse_workspace_bytes: the workspace a fuse() call of these sizes would
    allocate (0: none; queries <= 10,240 entries and <= 16 runs need none)."""
    return int(_lib.lib().qf_fuse_workspace_bytes(int(n_queries), int(n_retrievers),
                                                  int(max_entries), methods_mask(methods),
                                                  1 if needs_wide(max_entries) else 0))


def minmax_per_query(score: torch.Tensor, list_off: torch.Tensor, want_norm=True,
                     want_micro=True):
    require_device()
    n_lists = list_off.numel() - 1
    norm = torch.empty_like(score) if want_norm else None
    micro = torch.empty(score.shape, dtype=torch.int32, device=score.device) if want_micro else None
    _lib.call("qf_minmax_per_query", _ptr(score), _ptr(list_off), n_lists, _ptr(norm),
              _ptr(micro), _stream())
    return norm, micro


def minmax_colminmax(score: torch.Tensor, list_off: torch.Tensor, n_retrievers: int,
                     raw_qpp: torch.Tensor, want_norm=False, want_micro=True,
                     micro_out: Optional[torch.Tensor] = None,
                     mm_out: Optional[torch.Tensor] = None):
    """minmax_per_query + qpp_colminmax in one launch (an unsharded batch): returns
    (norm, micro, mm) — the same values as the two calls."""
    require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    dev = score.device
    norm = torch.empty_like(score) if want_norm else None
    micro = None
    if want_micro:
        micro = micro_out if micro_out is not None else torch.empty(score.shape, dtype=torch.int32,
                                                                    device=dev)
    mm = mm_out if mm_out is not None else torch.empty(2 * R * _lib.QPP_COLS,
                                                       dtype=torch.float64, device=dev)
    _lib.call("qf_minmax_colminmax", _ptr(score), _ptr(list_off), Q, R, _ptr(norm), _ptr(micro),
              _ptr(raw_qpp), _ptr(mm), _stream())
    return norm, micro, mm


def qpp_raw(score: torch.Tensor, list_off: torch.Tensor, n_retrievers: int, top_k: int,
            num_terms: torch.Tensor, text_feat: torch.Tensor,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    if out is None:
        out = torch.empty((Q * R, _lib.QPP_COLS), dtype=torch.float64, device=list_off.device)
    _lib.call("qf_qpp_raw", _ptr(score), _ptr(list_off), Q, R, int(top_k), _ptr(num_terms),
              _ptr(text_feat), _ptr(out), _stream())
    return out


def fused_topk(out: FuseOut, list_off: torch.Tensor, n_retrievers: int, k: int, dest=None):
    """qf_fused_topk: (docid int32 view of uint32 [Q, M, k], score float64 [Q, M, k]);
    rows shorter than k padded with docid 0xFFFFFFFF (-1) and NaN.  `dest`: a
    preallocated contiguous (docid, score) pair of that shape (dist.TopkGather's
    send buffers) to write into instead of new tensors."""
    dev = require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    M = out.fused.shape[0]
    if dest is not None:
        docid, score = dest
        if (tuple(docid.shape) != (Q, M, k) or tuple(score.shape) != (Q, M, k)
                or docid.dtype != torch.int32 or score.dtype != torch.float64
                or not (docid.is_contiguous() and score.is_contiguous())):
            raise ValueError(f"dest must be contiguous int32 / float64 [{Q}, {M}, {k}]")
    else:
        docid = torch.empty((Q, M, k), dtype=torch.int32, device=dev)
        score = torch.empty((Q, M, k), dtype=torch.float64, device=dev)
    _lib.call("qf_fused_topk_wide" if out.wide else "qf_fused_topk", Q, R, _ptr(list_off), _ptr(out.union_count), _ptr(out.union_docid),
              _ptr(out.perm), _ptr(out.fused), out.fused.shape[1], M, int(k), _ptr(docid),
              _ptr(score), _stream())
    return docid, score


def qpp_colminmax(raw: torch.Tensor, list_off: torch.Tensor, n_retrievers: int,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[2*R*13]: column minima then negated maxima (MIN all-reduce combines shards)."""
    require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    if out is None:
        out = torch.empty(2 * R * _lib.QPP_COLS, dtype=torch.float64, device=raw.device)
    _lib.call("qf_qpp_colminmax", _ptr(raw), _ptr(list_off), Q, R, _ptr(out), _stream())
    return out


def qpp_colmeanstd(raw: torch.Tensor, list_off: torch.Tensor, n_retrievers: int,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[2*R*13]: numpy's column means then stds (1.0 when not > 0), for zscore."""
    require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    if out is None:
        out = torch.empty(2 * R * _lib.QPP_COLS, dtype=torch.float64, device=raw.device)
    _lib.call("qf_qpp_colmeanstd", _ptr(raw), _ptr(list_off), Q, R, _ptr(out), _stream())
    return out


def qpp_normalize(raw: torch.Tensor, mm: Optional[torch.Tensor], list_off: torch.Tensor,
                  n_retrievers: int, mode: str = "minmax", qpp_index: int = 5,
                  want_norm=False, want_micro=True, want_weights=True) -> Dict[str, torch.Tensor]:
    require_device()
    R = int(n_retrievers)
    Q = (list_off.numel() - 1) // R
    dev = raw.device
    mode_id = {"none": _lib.NORM_NONE, "minmax": _lib.NORM_MINMAX,
               "zscore": _lib.NORM_ZSCORE}.get(mode)
    if mode_id is None:
        raise NotImplementedError(f"QPP normalisation '{mode}' is not implemented on device")
    norm = torch.empty_like(raw) if want_norm else None
    micro = torch.empty(raw.shape, dtype=torch.int64, device=dev) if want_micro else None
    w = torch.empty(Q * R, dtype=torch.float64, device=dev) if want_weights else None
    _lib.call("qf_qpp_normalize", _ptr(raw), _ptr(mm), _ptr(list_off), Q, R, mode_id,
              int(qpp_index), _ptr(norm), _ptr(micro), _ptr(w), _stream())
    return {"norm": norm, "micro": micro, "weights": w}


def qpp_features(micro: torch.Tensor, n_queries: int, n_retrievers: int, run_of_block,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qf_qpp_features: learned fusion's X [Q, 13 * len(run_of_block)] float64 from the
    normalised predictors' micro-units (qpp_normalize(..., want_micro=True))."""
    dev = require_device()
    blocks = np.ascontiguousarray(run_of_block, dtype=np.int32)
    Q, R = int(n_queries), int(n_retrievers)
    if micro.dtype != torch.int64 or micro.numel() != Q * R * _lib.QPP_COLS:
        raise ValueError(f"micro must be int64 [{Q * R}, {_lib.QPP_COLS}]")
    if out is None:
        out = torch.empty((Q, len(blocks) * _lib.QPP_COLS), dtype=torch.float64, device=dev)
    _lib.call("qf_qpp_features", _ptr(micro), Q, R, blocks.ctypes.data, len(blocks), _ptr(out),
              _stream())
    return out


def synth_runs_nq(q_begin: int, n_queries: int, n_retrievers: int, k: int, qrel_off=None,
                  qrel_doc=None, seed: int = 20251212, device=None):
    """SURVEY.md §8(d)'s synthetic runs on device (qf_synth_runs_nq): (list_off, docid,
    raw score).  qrel_off / qrel_doc: the judged documents to plant (CSR over qrel
    queries, corpus ids; numpy or device tensors), None = no planting."""
    import numpy as np
    dev = device or require_device()
    E = n_queries * n_retrievers * k
    list_off = torch.empty(n_queries * n_retrievers + 1, dtype=torch.int64, device=dev)
    docid = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
    score = torch.empty(max(E, 1), dtype=torch.float64, device=dev)
    qo = qd = None
    nq = 0
    if not 0 <= int(seed) < 2**32:  # Philox is keyed by a 32-bit seed (include/qppfuse.h)
        raise ValueError(f"synth_runs_nq: seed {seed} outside [0, 2**32)")
    if qrel_off is not None:
        # converted by value (an int64 docid array must not be reinterpreted as twice as
        # many int32 words); corpus ids are uint32, carried as int32 bits on device
        if isinstance(qrel_off, torch.Tensor):
            qo = qrel_off.to(device=dev, dtype=torch.int64)
        else:
            qo = torch.from_numpy(np.ascontiguousarray(qrel_off, dtype=np.int64)).to(dev)
        if isinstance(qrel_doc, torch.Tensor):
            qd = qrel_doc.to(device=dev)
            if qd.dtype != torch.int32:  # (int32: already the uint32 bits)
                qd = qd.to(torch.int64)
                if qd.numel() and (int(qd.min()) < 0 or int(qd.max()) >= 2**32):
                    raise ValueError("synth_runs_nq: qrel docids must fit uint32")
                qd = torch.where(qd >= 2**31, qd - 2**32, qd).to(torch.int32)
        else:
            d = np.asarray(qrel_doc)
            if d.size and (d.min() < 0 or d.max() >= 2**32):
                raise ValueError("synth_runs_nq: qrel docids must fit uint32")
            qd = torch.from_numpy(np.ascontiguousarray(d.astype(np.uint32)).view(np.int32)).to(dev)
        nq = qo.numel() - 1
        if int(qo[-1]) > qd.numel():
            raise ValueError("synth_runs_nq: qrel_off ends past qrel_doc")
    _lib.call("qf_synth_runs_nq", int(q_begin), int(n_queries), int(n_retrievers), int(k),
              int(seed), _ptr(qo), _ptr(qd), nq, _ptr(list_off), _ptr(docid),
              _ptr(score), _stream())
    return list_off, docid[:E], score[:E]


def synth_runs(q_begin: int, n_queries: int, n_retrievers: int, k: int, seed: int = 20251212,
               p_shared: float = 0.7, device=None):
    """Synthetic (list_off, docid, raw score) on device; see DESIGN.md."""
    dev = device or require_device()
    E = n_queries * n_retrievers * k
    list_off = torch.empty(n_queries * n_retrievers + 1, dtype=torch.int64, device=dev)
    docid = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
    score = torch.empty(max(E, 1), dtype=torch.float64, device=dev)
    _lib.call("qf_synth_runs", int(q_begin), int(n_queries), int(n_retrievers), int(k),
              int(seed) & (2**64 - 1), float(p_shared), _ptr(list_off), _ptr(docid), _ptr(score),
              _stream())
    return list_off, docid[:E], score[:E]


def gbdt_predict(X: torch.Tensor, packed) -> torch.Tensor:
    """qf_gbdt_predict: [n_rows, n_boosters] raw predictions (qppfuse.lgbm.PackedModel)."""
    dev = require_device()
    if X.dtype != torch.float64 or X.dim() != 2 or X.shape[1] != packed.n_features:
        raise ValueError(f"X must be float64 [n, {packed.n_features}]")
    d = packed.to_device(dev)
    out = torch.empty((X.shape[0], packed.n_boosters), dtype=torch.float64, device=dev)
    _lib.call("qf_gbdt_predict", X.shape[0], _ptr(X.contiguous()), packed.n_features,
              packed.n_boosters, _ptr(d["tree_off"]), _ptr(d["node_off"]), _ptr(d["leaf_off"]),
              _ptr(d["feature"]), _ptr(d["threshold"]), _ptr(d["dtype"]), _ptr(d["left"]),
              _ptr(d["right"]), _ptr(d["leaf_value"]), _ptr(out), _stream())
    return out


def learned_gbdt_weights(micro: Optional[torch.Tensor], n_queries: int, n_retrievers: int,
                         run_of_block, packed, run_to_booster, want_pred: bool = False,
                         raw_qpp: Optional[torch.Tensor] = None, mm: Optional[torch.Tensor] = None,
                         list_off: Optional[torch.Tensor] = None, mode: str = "minmax"):
    """qf_learned_gbdt_weights: qpp_features + gbdt_predict + learned_weights in one
    launch — [Q * R] run weights (and the raw [Q, B] predictions if want_pred).  The
    features come from `micro` (qpp_normalize's micro-units) or, with micro None,
    from raw_qpp normalised on the fly with mm (qpp_colminmax / qpp_colmeanstd) —
    the normalisation launch folded in.  For models of up to 19 retrievers (13
    features each); bit-identical to the separate calls."""
    import numpy as np
    dev = require_device()
    Q, R = int(n_queries), int(n_retrievers)
    blocks = np.ascontiguousarray(run_of_block, dtype=np.int32)
    rb = np.ascontiguousarray(run_to_booster, dtype=np.int32)
    mode_id = {"none": _lib.NORM_NONE, "minmax": _lib.NORM_MINMAX,
               "zscore": _lib.NORM_ZSCORE}[mode]
    if micro is None:
        if raw_qpp is None or list_off is None or (mode_id != _lib.NORM_NONE and mm is None):
            raise ValueError("raw_qpp, list_off (and mm) are needed without micro")
        if raw_qpp.dtype != torch.float64 or raw_qpp.numel() != Q * R * _lib.QPP_COLS:
            raise ValueError(f"raw_qpp must be float64 [{Q * R}, {_lib.QPP_COLS}]")
    elif micro.dtype != torch.int64 or micro.numel() != Q * R * _lib.QPP_COLS:
        raise ValueError(f"micro must be int64 [{Q * R}, {_lib.QPP_COLS}]")
    if packed.n_features != len(blocks) * _lib.QPP_COLS:
        raise ValueError("the model's features must be 13 per block of run_of_block")
    d = packed.to_device(dev)
    w = torch.empty(Q * len(rb), dtype=torch.float64, device=dev)
    pred = torch.empty((Q, packed.n_boosters), dtype=torch.float64, device=dev) if want_pred else None
    _lib.call("qf_learned_gbdt_weights", Q, _ptr(None if micro is None else micro.contiguous()),
              _ptr(raw_qpp), _ptr(mm), _ptr(list_off), mode_id, R, blocks.ctypes.data,
              len(blocks), packed.n_boosters, _ptr(d["tree_off"]), _ptr(d["node_off"]),
              _ptr(d["leaf_off"]), _ptr(d["feature"]), _ptr(d["threshold"]), _ptr(d["dtype"]),
              _ptr(d["left"]), _ptr(d["right"]), _ptr(d["leaf_value"]), len(rb), rb.ctypes.data,
              _ptr(pred), _ptr(w), _stream())
    return (w, pred) if want_pred else w


def learned_weights(pred: torch.Tensor, run_to_booster) -> torch.Tensor:
    """qf_learned_weights: [Q * R] run weights from [Q, B] predictions."""
    import numpy as np
    dev = require_device()
    rb = np.ascontiguousarray(run_to_booster, dtype=np.int32)
    Q, B = pred.shape
    w = torch.empty(Q * len(rb), dtype=torch.float64, device=dev)
    _lib.call("qf_learned_weights", Q, _ptr(pred.contiguous()), B, len(rb), rb.ctypes.data,
              _ptr(w), _stream())
    return w


def mlp_weights(X: torch.Tensor, model, run_to_output) -> torch.Tensor:
    """qf_mlp_weights: [Q * R] float32 FusionMLP run weights (as float64) from
    learned_fusion's feature matrix X [Q, n_qpp * n_retrievers] (qppfuse.mlp.MLPModel)."""
    import numpy as np
    dev = require_device()
    if X.dtype != torch.float64 or X.dim() != 2:
        raise ValueError("X must be float64 [n_queries, n_qpp * n_retrievers]")
    cols = model.input_columns()
    if cols.size and int(cols.max()) >= X.shape[1]:
        raise ValueError(f"the model reads column {int(cols.max())} of a {X.shape[1]}-column X")
    d = model.to_device(dev)
    widths = np.ascontiguousarray(model.widths(), dtype=np.int32)
    ro = np.ascontiguousarray(run_to_output, dtype=np.int32)
    Q = X.shape[0]
    w = torch.empty(max(Q * len(ro), 1), dtype=torch.float64, device=dev)
    _lib.call("qf_mlp_weights", Q, _ptr(X.contiguous()), X.shape[1], _ptr(d["in_col"]),
              len(widths) - 1, widths.ctypes.data, _ptr(d["params"]), len(ro), ro.ctypes.data,
              _ptr(w), _stream())
    return w[:Q * len(ro)]

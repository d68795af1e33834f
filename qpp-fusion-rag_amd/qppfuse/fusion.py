"""Drop-in replacement for the reference's src/fusion.py, computed on MI355X.

Same public names, signatures, return shapes and exceptions as
PoisedDok/QPP-Fusion-RAG src/fusion.py (imported by scripts/05_fusion.py:40-53):
load_runs, load_qpp_scores, get_qpp_weight, get_qpp_index, combsum, combmnz,
rrf, weighted_combsum, weighted_combmnz, weighted_rrf, learned_fusion,
write_runfile, run_fusion.

What changes is where the work happens: the runs are packed once into CSR
columns (qppfuse.runset), uploaded to HBM, and every requested method is
computed for every query by one launch of the HIP kernel qf_fuse
(csrc/qf_fuse.hip).  Results come back as a FusedRun — a read-only Mapping
{qid: [(docno, score), ...]} that materialises lists on access — in the order
the reference returns them: score-descending for combsum/combmnz/rrf (ranx +
_ranx_to_dict, src/fusion.py:469-477), first-seen order for the weighted
methods (src/fusion.py:278-279), docno order for learned_fusion (its pandas
groupby, src/fusion.py:443-446).
"""
from __future__ import annotations

import os
import threading
import weakref
from collections.abc import Mapping
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd

from . import _lib, engine
from .config import ConfigError, config
from .config import get_qpp_index as _cfg_qpp_index
from .data_utils import load_qpp_scores as _load_qpp
from .runset import RunSet, dedupe_keep_last, expand_duplicates, pack_frames, reorder

__all__ = ["load_runs", "load_qpp_scores", "get_qpp_weight", "get_qpp_index", "combsum",
           "combmnz", "rrf", "weighted_combsum", "weighted_combmnz", "weighted_rrf",
           "learned_fusion", "write_runfile", "run_fusion", "fuse_many", "FusedRun",
           "ConfigError"]

UNWEIGHTED = ("combsum", "combmnz", "rrf")
WEIGHTED = ("wcombsum", "wcombmnz", "wrrf")


# ------------------------------------------------------------------ loading --

def load_runs(res_path: str, use_normalized: bool = True) -> Dict[str, pd.DataFrame]:
    """{ranker: DataFrame[qid, iter, docno, rank, score, runid]} in os.listdir order.

    Parsed natively (qppfuse.fastio, csrc/qf_io.cpp) into the packed run set the
    kernels read — cached for these frames, so the fusions skip packing.  The
    string columns hold the interned str objects (dtype object, as pandas reads
    them in the reference)."""
    from . import fastio
    suffix = ".norm.res" if use_normalized else ".res"
    files = [f for f in os.listdir(res_path) if f.endswith(suffix)]
    if not files:
        raise FileNotFoundError(f"No {suffix} files found in {res_path}")
    names = [f.replace(suffix, "") for f in files]
    rs, frames = fastio.parse_runs([os.path.join(res_path, f) for f in files], names)
    _remember(frames, rs)
    return frames


def load_qpp_scores(qpp_path: str) -> Dict[str, Dict[str, List[float]]]:
    return _load_qpp(qpp_path)


def get_qpp_weight(qid: str, ranker: str, qpp_data, qpp_index: int = None,
                   fusion_mode: bool = False) -> float:
    """Weight of (query, ranker); KeyError / IndexError exactly where the reference raises."""
    if qpp_index is None:
        qpp_index = config.qpp.default_index
    if qid not in qpp_data:
        raise KeyError(f"QPP data missing for query '{qid}'. Run QPP computation first.")
    if ranker not in qpp_data[qid]:
        raise KeyError(f"QPP data missing for ranker '{ranker}' on query '{qid}'. "
                       f"Available: {list(qpp_data[qid].keys())}")
    vals = qpp_data[qid][ranker]
    if fusion_mode or qpp_index == -1:
        return sum(vals) / len(vals)
    if qpp_index >= len(vals):
        raise IndexError(f"QPP index {qpp_index} out of range. Available: 0-{len(vals)-1}")
    return vals[qpp_index]


def get_qpp_index(model_name: str) -> int:
    return _cfg_qpp_index(model_name)


# --------------------------------------------------------------- results -----

def qid_sort_key(x: str):
    """write_runfile's qid order (src/fusion.py:487); mixed kinds raise TypeError."""
    return int(x.replace("test", "")) if x.startswith("test") else x


class FusedRun(Mapping):
    """{qid: [(docno, score)]} backed by the kernel's packed output arrays: per query
    (at qbase), the union's docids and fused scores in first-seen order, and perm,
    the first-seen indices in rank order (include/qppfuse.h)."""

    def __init__(self, qids, docnos, qbase, counts, union_docid, perm, fused, order: str,
                 runset: Optional[RunSet] = None):
        self._rs = runset
        self._qids = list(qids)
        self._index = {q: i for i, q in enumerate(self._qids)}
        self._docnos = docnos
        self._qbase = qbase
        self._counts = counts
        self._udoc = union_docid
        self._perm = perm
        self._fused = fused
        self.order = order  # "sorted", "first_seen" or "docno"

    def __len__(self):
        return len(self._qids)

    def __iter__(self):
        return iter(self._qids)

    def __contains__(self, qid):
        return qid in self._index

    def arrays(self, qid) -> Tuple[np.ndarray, np.ndarray]:
        """(docno ids, scores) of one query in score-descending order."""
        i = self._index[qid]
        b, n = int(self._qbase[i]), int(self._counts[i])
        p = self._perm[b:b + n].astype(np.int64)
        return self._udoc[b + p], self._fused[b + p]

    def __getitem__(self, qid) -> List[Tuple[str, float]]:
        i = self._index[qid]
        b, n = int(self._qbase[i]), int(self._counts[i])
        if self.order == "sorted":
            p = self._perm[b:b + n].astype(np.int64)
            docs = self._docnos[self._udoc[b + p]]
            return list(zip(docs.tolist(), self._fused[b + p].tolist()))
        by_u = self._fused[b:b + n]
        ids = self._udoc[b:b + n]
        if self.order == "docno":  # ids are interned in docno order
            o = np.argsort(ids, kind="stable")
            ids, by_u = ids[o], by_u[o]
        docs = self._docnos[ids]
        return list(zip(docs.tolist(), by_u.tolist()))

    def to_dict(self) -> Dict[str, List[Tuple[str, float]]]:
        return {q: self[q] for q in self._qids}


# ---------------------------------------------------------------- packing ----

_PACK_CACHE: Dict[tuple, tuple] = {}  # frames' identity -> (content fingerprint, RunSet)


class _Pinned:
    """A column digest that also holds what it hashed; equal when the digests are."""
    __slots__ = ("h", "ref")

    def __init__(self, h, ref):
        self.h, self.ref = h, ref

    def __eq__(self, other):
        return isinstance(other, _Pinned) and other.h == self.h

    def __hash__(self):
        return self.h


def _column_digest(col):
    """xxh3 of one column's contents: the values of a numeric column, the object
    pointers of an object column (str objects are immutable, so an unchanged
    pointer is an unchanged value; any assignment into the column changes it);
    an Arrow-backed column by its (immutable) array."""
    import ctypes
    import xxhash
    pa_arr = getattr(col.array, "_pa_array", None)
    if pa_arr is not None:
        # Arrow-backed (load_runs' string columns): Arrow arrays are immutable and
        # pandas replaces the array on any assignment, so the array object itself
        # identifies the contents (held here, so its id cannot be reused)
        return ("arrow", id(pa_arr), pa_arr)
    a = np.ascontiguousarray(col.to_numpy())
    if a.dtype == object:
        if len(a) == 0:
            return 0
        # pinned: a copy of the column's references keeps every hashed str alive,
        # so no later value can reuse one of these addresses (A -> B -> C at A's
        # address would otherwise fingerprint as unchanged)
        a = a.copy()
        ptrs = (ctypes.c_uint64 * len(a)).from_address(a.ctypes.data)
        h = xxhash.xxh3_64_intdigest(memoryview(ptrs).cast("B"))
        del ptrs
        return _Pinned(h, a)
    if a.nbytes >= (1 << 22):  # large numeric columns: hashed over the threads
        from . import fastio
        return ("n", a.dtype.str, fastio.hash_bytes(a))
    return xxhash.xxh3_64_intdigest(memoryview(a).cast("B"))


def _fingerprint(runs: Dict[str, pd.DataFrame]) -> tuple:
    """Content of every column the fusions read (qid, docno, rank, score)."""
    return tuple((name, len(df), tuple(_column_digest(df[c]) for c in ("qid", "docno", "rank",
                                                                       "score")))
                 for name, df in runs.items())


def _key(runs: Dict[str, pd.DataFrame]) -> tuple:
    return tuple((name, id(df)) for name, df in runs.items())


def _remember(runs: Dict[str, pd.DataFrame], rs: RunSet) -> None:
    key = _key(runs)
    _PACK_CACHE.clear()
    _PACK_CACHE[key] = (_fingerprint(runs), rs)
    for df in runs.values():
        weakref.finalize(df, _PACK_CACHE.pop, key, None)


def _pack(runs: Dict[str, pd.DataFrame]) -> RunSet:
    """Pack once per runs dict: cached while the frames live AND their contents are
    unchanged (a frame edited in place is packed again — the reference is stateless)."""
    hit = _PACK_CACHE.get(_key(runs))
    if hit is not None and hit[0] == _fingerprint(runs):
        return hit[1]
    rs = pack_frames(runs)
    _remember(runs, rs)
    return rs


def _derived(rs: RunSet, what: str) -> RunSet:
    """The run set in the order / shape one method family reads (cached on rs)."""
    cache = rs.__dict__.setdefault("_derived_sets", {})
    if what not in cache:
        if what == "ranx":        # {docno: score} per list, score-sorted (src/fusion.py:459-465)
            d = dedupe_keep_last(rs)
            cache[what] = d if d.canonical else reorder(d, "score")
        elif what == "rows":      # every row, file order (src/fusion.py:272-277)
            cache[what] = _check_runs(rs, expand_duplicates(rs))
        elif what == "rank":      # every row, rank order (src/fusion.py:372)
            cache[what] = _check_runs(rs, expand_duplicates(rs if rs.canonical
                                                           else reorder(rs, "rank")))
        else:
            raise ValueError(what)
    return cache[what]


def _check_runs(rs: RunSet, rv: RunSet) -> RunSet:
    """A docno repeated d times inside one list becomes d virtual runs of its
    ranker: say so when that takes the run set past the kernels' 32 runs."""
    if rv.n_rankers > _lib.MAX_RUNS:
        depth = int(np.bincount(rv.base_ranker).max()) if rv.base_ranker is not None else 1
        raise ValueError(
            f"{rs.n_rankers} runs with docnos repeated up to {depth} times inside one list "
            f"expand to {rv.n_rankers} runs (every repeated row is summed as the reference's "
            f"loops sum it); at most {_lib.MAX_RUNS} are supported")
    return rv


def _expand_weights(weights: Optional[np.ndarray], rs: RunSet, rv: RunSet):
    if weights is None or rv.base_ranker is None or rv is rs:
        return weights
    return np.ascontiguousarray(weights.reshape(rs.n_queries, rs.n_rankers)[:, rv.base_ranker]
                                .ravel())


def _weights(rs: RunSet, qpp_data, qpp_index: int) -> np.ndarray:
    """[Q*R] weights in the reference's visiting order, raising as it does."""
    fusion_mode = qpp_index == -1
    n = rs.n_queries * rs.n_rankers
    try:  # every lookup present: one comprehension instead of a call per (qid, ranker)
        if fusion_mode:
            it = (sum(v) / len(v) for q in rs.qids for v in map(qpp_data[q].__getitem__, rs.rankers))
        else:
            it = (qpp_data[q][r][qpp_index] for q in rs.qids for r in rs.rankers)
        return np.fromiter(it, dtype=np.float64, count=n)
    except (KeyError, IndexError, TypeError, ValueError, ZeroDivisionError):
        pass  # the loop below raises what the reference raises, where it raises it
    w = np.empty(n, dtype=np.float64)
    k = 0
    for qid in rs.qids:
        for ranker in rs.rankers:
            w[k] = get_qpp_weight(qid, ranker, qpp_data, qpp_index, fusion_mode)
            k += 1
    return w


def _launch(rs: RunSet, methods: Sequence[str], rrf_k: int, weights: Optional[np.ndarray],
            learned_f32: Optional[int] = None):
    import torch
    engine.require_device()
    d = rs.to_device()
    if weights is None or isinstance(weights, torch.Tensor):
        wd = weights
    else:
        wd = torch.from_numpy(weights).to(d["list_off"].device)
    out = engine.fuse(d["list_off"], d["docid"], d["score"], rs.n_rankers, list(methods),
                      rrf_k=rrf_k, weights=wd, rank=d["rank"], max_entries=rs.max_entries(),
                      learned_f32=learned_f32)
    counts = out.union_count.cpu().numpy()[:rs.n_queries]
    bad = np.nonzero(counts < 0)[0]
    if bad.size:
        from ._lib import QF_QSTATUS
        code = int(counts[bad[0]])
        raise ValueError(f"query '{rs.qids[bad[0]]}': {QF_QSTATUS.get(code, code)}")
    E = rs.n_entries
    qbase = rs.query_base()
    total = int(counts.sum())
    if 0 < total < E:
        # only the unions cross PCIe: query q's U_q slots of every output, gathered
        # on the device into consecutive ranges (C2: 0.55 GB instead of 1.1 GB);
        # perm holds union positions, so it is unchanged
        dev = out.union_count.device
        cnt = torch.from_numpy(counts.astype(np.int64)).to(dev)
        cb = torch.cumsum(cnt, 0) - cnt  # compact base of each query
        qb = torch.from_numpy(np.ascontiguousarray(qbase, np.int64)).to(dev)
        q_of = torch.repeat_interleave(torch.arange(len(counts), device=dev), cnt,
                                       output_size=total)
        idx = qb[q_of] + (torch.arange(total, device=dev) - cb[q_of])
        # into pinned host buffers (torch's caching host allocator keeps them for the
        # next call) while the live pinned copy-backs stay under a cap, pageable
        # beyond it; the copies queued, one synchronisation
        hosts = [_host_copy(t) for t in (out.union_docid[idx], out.perm[:, idx],
                                         out.fused[:, idx], cb)]
        torch.cuda.current_stream(dev).synchronize()
        udoc = hosts[0].view(np.uint32)
        perm = hosts[1].view(np.uint32 if out.wide else np.uint16)
        fused = hosts[2]
        qbase = hosts[3]
    else:
        udoc = out.union_docid.cpu().numpy()[:E].view(np.uint32)
        perm = out.perm.cpu().numpy()[:, :E].view(np.uint32 if out.wide else np.uint16)
        fused = out.fused.cpu().numpy()[:, :E]
    res = {}
    for m, name in enumerate(out.methods):
        order = ("sorted" if name in UNWEIGHTED else "docno" if name == "learned"
                 else "first_seen")
        res[name] = FusedRun(rs.qids, rs.docnos, qbase, counts, udoc, perm[m],
                             fused[m], order, rs)
    return res


# Page-locked bytes held by live FusedRuns (their numpy views keep the host tensors
# alive).  A FusedRun's arrays are pinned while the live total stays under the cap
# (QPPFUSE_PINNED_CAP_MB, default 4096): pinned pages cannot be swapped, and
# workflows that keep many runs alive (argmax_runs' 13 QPP-column runs, experiment)
# would otherwise grow page-locked memory without bound.  Beyond the cap the
# copy-back lands in pageable memory (~5x slower, same bytes).  The cap counts LIVE
# bytes; torch's caching host allocator also keeps FREED pinned blocks for reuse, so
# when a copy-back would cross the cap that cache is emptied first
# (torch._C._host_emptyCache: blocks no live tensor holds go back to the OS) — the
# page-locked total then stays within the cap plus what the allocator caches between
# two such crossings.  The counter is updated under a lock (FusedRuns may be built
# and dropped on several threads).
_PINNED = {"live": 0}
_PINNED_LOCK = threading.Lock()


def _pinned_cap() -> int:
    return int(os.environ.get("QPPFUSE_PINNED_CAP_MB", "4096")) << 20


def _release_pinned(nbytes: int) -> None:
    with _PINNED_LOCK:
        _PINNED["live"] -= nbytes


def _host_copy(t) -> np.ndarray:
    """Device tensor -> host numpy array (pinned when under the cap: ~5x faster
    copy-back); a finalizer returns the pinned bytes when the array is no longer
    alive (a tensor's .numpy() holds its storage, not the tensor)."""
    import torch
    nbytes = t.numel() * t.element_size()
    with _PINNED_LOCK:
        pinned = _PINNED["live"] + nbytes <= _pinned_cap()
        if pinned:
            _PINNED["live"] += nbytes
        elif hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()  # the cached, freed pinned blocks
    try:
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=pinned)
    except BaseException:
        if pinned:
            _release_pinned(nbytes)
        raise
    h.copy_(t, non_blocking=True)  # pageable: the runtime stages it
    a = h.numpy()
    if pinned:
        weakref.finalize(a, _release_pinned, nbytes)
    return a


def pinned_bytes_live() -> int:
    """Page-locked bytes the live FusedRuns hold (see _PINNED)."""
    return _PINNED["live"]


def fuse_many(runs: Dict[str, pd.DataFrame], methods: Sequence[str], qpp_data=None,
              qpp_index: Optional[int] = None, k: Optional[int] = None) -> Dict[str, FusedRun]:
    """Several methods from one packed upload (one launch when the lists are canonical)."""
    methods = [m.lower() for m in methods]
    k = k if k is not None else config.fusion.rrf_k
    qpp_index = qpp_index if qpp_index is not None else config.qpp.default_index
    rs = _pack(runs)
    weighted = [m for m in methods if m in WEIGHTED]
    weights = _weights(rs, qpp_data, qpp_index) if weighted else None
    if rs.canonical and not rs.has_dups:
        return _launch(rs, methods, k, weights)
    # Lists whose file order is not score order, or with a docno repeated inside
    # one list: each family gets the lists the reference iterates (ranx:
    # {docno: score}, last row wins, score-sorted; W-CombSUM/MNZ: every row in
    # file order; W-RRF: every row in rank order, src/fusion.py:372).
    res = {}
    un = [m for m in methods if m in UNWEIGHTED]
    if un:
        res.update(_launch(_derived(rs, "ranx"), un, k, None))
    ws = [m for m in methods if m in ("wcombsum", "wcombmnz")]
    if ws:
        rv = _derived(rs, "rows")
        res.update(_launch(rv, ws, k, _expand_weights(weights, rs, rv)))
    if "wrrf" in methods:
        rv = _derived(rs, "rank")
        res.update(_launch(rv, ["wrrf"], k, _expand_weights(weights, rs, rv)))
    return {m: res[m] for m in methods}


# ------------------------------------------------------- public fusions ------

def combsum(runs: Dict[str, pd.DataFrame]) -> FusedRun:
    """CombSUM(d,q) = Σ_i S_i(d,q) over min-max normalised runs (ranx "sum")."""
    return fuse_many(runs, ["combsum"])["combsum"]


def combmnz(runs: Dict[str, pd.DataFrame]) -> FusedRun:
    """CombMNZ(d,q) = |{i: d ∈ R_i}| · Σ_i S_i(d,q) (ranx "mnz")."""
    return fuse_many(runs, ["combmnz"])["combmnz"]


def rrf(runs: Dict[str, pd.DataFrame], k: int = None) -> FusedRun:
    """RRF(d,q) = Σ_i 1/(k + rank_i(d,q)) (ranx "rrf"), k from config when None."""
    return fuse_many(runs, ["rrf"], k=k)["rrf"]


def weighted_combsum(runs, qpp_data, qpp_index: int = None) -> FusedRun:
    """W-CombSUM(d,q) = Σ_i w_i(q) · S_i(d,q); qpp_index -1 = mean of the 13 columns."""
    return fuse_many(runs, ["wcombsum"], qpp_data, qpp_index)["wcombsum"]


def weighted_combmnz(runs, qpp_data, qpp_index: int = None) -> FusedRun:
    """W-CombMNZ(d,q) = |{i}| · Σ_i w_i(q) · S_i(d,q)."""
    return fuse_many(runs, ["wcombmnz"], qpp_data, qpp_index)["wcombmnz"]


def weighted_rrf(runs, qpp_data, qpp_index: int = None, k: int = None) -> FusedRun:
    """W-RRF(d,q) = Σ_i w_i(q) / (k + rank_i(d,q)) with the file's rank column."""
    return fuse_many(runs, ["wrrf"], qpp_data, qpp_index, k)["wrrf"]


def learned_fusion(runs: Dict[str, pd.DataFrame], qpp_data, model_path: str,
                   retrievers: Optional[List[str]] = None) -> FusedRun:
    """Fusion with per-query weights from a learned model (src/fusion.py:387-448).

    The model pickle is read statically (qppfuse.lgbm / qppfuse.mlp: no
    unpickling).  LightGBM (MultiOutputLGBM / PerRetrieverLGBM): the 13·R QPP
    features go through the boosters on device (qf_gbdt_predict) and are
    normalised as BaseFusionModel._normalize_weights does (qf_learned_weights).
    FusionMLP: the selected QPP columns go through the MLP, softmax and the same
    normalisation in float32 (qf_mlp_weights), and the row products are float32
    as numpy 2 forms row["score"] * np.float32 (qf_fuse_learned_f32).  Then
    qf_fuse(QF_LEARNED) forms Σ score·w per document in pandas' groupby-sum order.
    Lists come back in docno order, as the reference's groupby returns them."""
    import torch
    from . import lgbm, mlp
    print(f"[fusion] Running learned fusion from {model_path}...")
    key = (os.path.abspath(model_path), os.path.getmtime(model_path))
    cached = _MODELS.get(key)
    if cached is None:
        if mlp.model_kind(model_path) == "FusionMLP":
            cached = (mlp.load_mlp_model(model_path), None)
        else:
            model = lgbm.load_fusion_model(model_path)
            cached = (model, lgbm.pack_model(model))
        _MODELS[key] = cached
    model, packed = cached
    is_mlp = packed is None
    retrievers = list(retrievers or model.retrievers)
    n_qpp = model.n_qpp
    n_out = model.n_outputs if is_mlp else len(model.boosters)
    if len(retrievers) != n_out:
        raise ValueError(f"the model predicts {n_out} weights but "
                         f"{len(retrievers)} retrievers were given")
    rs = _pack(runs)
    Q = rs.n_queries
    X = np.zeros((Q, n_qpp * len(retrievers)))  # src/fusion.py:421-427
    for i, qid in enumerate(rs.qids):
        qd = qpp_data.get(qid)
        if qd is None:
            continue
        for j, retriever in enumerate(retrievers):
            if retriever in qd:
                X[i, j * n_qpp:(j + 1) * n_qpp] = qd[retriever][:n_qpp]
    dev = engine.require_device()
    # a docno repeated inside one list adds every row (the groupby sum,
    # src/fusion.py:440-441): repeated rows go to virtual runs of their ranker
    rv = _derived(rs, "rows")
    names = [rs.rankers[b] for b in rv.base_ranker] if rv.base_ranker is not None else rs.rankers
    run_to_out = [retrievers.index(r) if r in retrievers else -1 for r in names]
    Xd = torch.from_numpy(X).to(dev)
    if is_mlp:
        w = engine.mlp_weights(Xd, model, run_to_out)
        f32 = sum(1 << r for r, j in enumerate(run_to_out) if j >= 0)
        res = _launch(rv, ["learned"], config.fusion.rrf_k, w, learned_f32=f32)
    else:
        w = engine.learned_weights(engine.gbdt_predict(Xd, packed), run_to_out)
        res = _launch(rv, ["learned"], config.fusion.rrf_k, w)
    fused = res["learned"]
    print(f"[fusion] Learned fusion done: {len(fused)} queries")
    return fused


_MODELS: Dict[tuple, tuple] = {}  # (path, mtime) -> (FusionModel, PackedModel) | (MLPModel, None)


# ------------------------------------------------------------------ output ---

def write_runfile(fused: Mapping, output_path: str, tag: str = "fusion") -> None:
    """TREC run file: qids by qid_sort_key, docs by score desc (stable), '%.6f' scores.

    A FusedRun is written by the native writer (qppfuse.fastio: csrc/qf_io.cpp)
    straight from the kernel's ranked arrays; any other mapping as the
    reference does it."""
    if isinstance(fused, FusedRun) and fused._rs is not None:
        write_fused_native(fused, output_path, tag)
        print(f"Wrote fused run to {output_path}")
        return
    with open(output_path, "w") as fout:
        for qid in sorted(fused.keys(), key=qid_sort_key):
            ranked = sorted(fused[qid], key=lambda x: x[1], reverse=True)
            fout.write("".join(f"{qid} Q0 {d} {i} {s:.6f} {tag}\n"
                               for i, (d, s) in enumerate(ranked, start=1)))
    print(f"Wrote fused run to {output_path}")


def write_fused_native(fused: "FusedRun", output_path: str, tag: str, select=None,
                       rename=None) -> None:
    """write_runfile of a FusedRun, optionally of the queries `select(qid)` keeps,
    written under `rename(qid)` (multicorpus: one corpus, bare qids)."""
    from . import fastio
    qids = [q for q in fused.keys() if select is None or select(q)]
    names = {q: (rename(q) if rename else q) for q in qids}
    idx = fused._index
    order = np.asarray([idx[q] for q in sorted(qids, key=lambda q: qid_sort_key(names[q]))],
                       np.int64)
    qid_table = None
    if rename is not None:
        enc = [(rename(q) if (select is None or select(q)) else q).encode() for q in fused._qids]
        off = np.zeros(len(enc) + 1, np.int64)
        np.cumsum([len(e) for e in enc], out=off[1:])
        qid_table = (off, b"".join(enc))
    fastio.write_run(output_path, order, fused._qbase, fused._counts, fused._udoc,
                     fused._perm, fused._fused, fused._rs, tag, qid_table=qid_table)


def run_fusion(method: str, runs_dir: str, qpp_dir: Optional[str] = None, qpp_model: str = None,
               model_path: Optional[str] = None, output_path: Optional[str] = None,
               rrf_k: int = None):
    """Load, fuse with one method, optionally write — same dispatch and tags as the reference."""
    qpp_model = qpp_model or config.qpp.default_method
    rrf_k = rrf_k if rrf_k is not None else config.fusion.rrf_k
    runs = load_runs(runs_dir, use_normalized=True)
    print(f"Loaded {len(runs)} rankers: {list(runs.keys())}")
    method = method.lower()
    if method in ("combsum", "combmnz"):
        fused, tag = fuse_many(runs, [method])[method], method
    elif method == "rrf":
        fused, tag = rrf(runs, k=rrf_k), f"rrf-k{rrf_k}"
    elif method in ("wcombsum", "w-combsum", "wcombmnz", "w-combmnz", "wrrf", "w-rrf"):
        if not qpp_dir:
            raise ValueError("--qpp_dir required for weighted methods")
        name = method.replace("-", "")
        qpp_data = load_qpp_scores(qpp_dir)
        qpp_index = get_qpp_index(qpp_model)
        fused = fuse_many(runs, [name], qpp_data, qpp_index, rrf_k)[name]
        tag = f"{name}-{qpp_model.lower()}"
    elif method == "learned":
        if not model_path:
            raise ValueError("--model_path required for learned fusion")
        if not qpp_dir:
            raise ValueError("--qpp_dir required for learned fusion")
        fused, tag = learned_fusion(runs, load_qpp_scores(qpp_dir), model_path), "learned"
    else:
        raise ValueError(f"Unknown method '{method}'. Valid: {config.fusion.methods}")
    if output_path:
        write_runfile(fused, output_path, tag)
    return fused

"""Drop-in replacement for the reference's src/qpp.py, computed on MI355X.

The reference computes the 13 QPP predictors in a JVM subprocess
(QPPBridge.java, fed JSON over stdin, src/qpp.py:117-171).  Here the same
predictors are a HIP kernel (csrc/qf_qpp.hip, one wavefront per ranked list);
the per-column normalisation (minmax / zscore) and the "%.6f" write-back are
kernels too.
Public surface kept: QPPResult, QPPBridge (compute_batch / compute),
compute_qpp_for_res_file, _normalize_qpp — same arguments, return values,
output files and exception types (RuntimeError when the engine is unavailable,
FileNotFoundError / ValueError on bad inputs).
"""
from __future__ import annotations

import json
import os
import sys
import time
from collections import defaultdict
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import numpy as np

from . import _lib, engine, textfeat
from .config import QPP_METHODS as JAVA_METHODS
from .config import config

# The names QPPBridge.java emits, in its output order (QPPBridge.java:148-188);
# also the column order of the raw predictor kernel qf_qpp_raw.
QPP_METHODS = list(JAVA_METHODS)


@dataclass
class QPPResult:
    query: str
    retriever_name: str
    qpp_scores: Dict[str, float]
    methods_used: List[str]
    processing_time_ms: float
    predictions: Dict[str, Any]
    error: Optional[str] = None


def _round_f32_exact(q) -> float:
    """The float32 nearest the rational q (ties to even), as a Python float."""
    from fractions import Fraction
    if q == 0:
        return 0.0
    neg = q < 0
    a = -q if neg else q
    # a = m * 2^e with m in [2^23, 2^24): e from the bit lengths, then round m
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    e = max(e - 23, -149)  # float32 subnormals: a fixed exponent of 2^-149
    m = a / Fraction(2) ** e
    fl = m.numerator // m.denominator
    rem = m - fl
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and fl % 2 == 1):
        fl += 1
    v = float(fl) * 2.0 ** e
    if v > float(np.finfo(np.float32).max):
        v = float("inf")
    return -v if neg else v


def java_floats(x: np.ndarray) -> np.ndarray:
    """What QPPBridge.java holds for each double the reference sends it: Python's
    json.dumps writes repr(v) (the shortest decimal that round-trips), Gson's
    getAsFloat is Float.parseFloat of that text (QPPBridge.java:67-70, src/qpp.py:
    130-147) — one correct rounding of the DECIMAL.  The kernel rounds the double
    (RN-even); the two differ only when the double lies exactly halfway between two
    floats and its shortest decimal is not that midpoint, so those values (and any
    outside the float normal range) are replaced here by the float Java reads, held
    as a double (which the kernel then converts exactly)."""
    from fractions import Fraction
    x = np.ascontiguousarray(x, dtype=np.float64)
    bits = x.view(np.uint64)
    exp = (bits >> np.uint64(52)) & np.uint64(0x7FF)
    normal32 = (exp >= np.uint64(1023 - 126)) & (exp <= np.uint64(1023 + 127))
    midpoint = (bits & np.uint64(0x1FFFFFFF)) == np.uint64(0x10000000)
    fix = np.nonzero((midpoint | ~normal32) & np.isfinite(x) & (x != 0.0))[0]
    if fix.size == 0:
        return x
    out = x.copy()
    for i in fix:
        out[i] = _round_f32_exact(Fraction(repr(float(x[i]))))
    return out


def _device_qpp(lists: List[List[float]], texts: List[str], top_k: int = 0) -> np.ndarray:
    """Raw predictors [L, 13] for L score lists (each used in the given order)."""
    lens = np.fromiter((len(s) for s in lists), dtype=np.int64, count=len(lists))
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    flat = np.fromiter((float(x) for s in lists for x in s), dtype=np.float64, count=int(off[-1]))
    return _device_qpp_flat(flat, off, texts, top_k)


def _device_qpp_flat(flat: np.ndarray, off: np.ndarray, texts: List[str],
                     top_k: int = 0) -> np.ndarray:
    """Raw predictors [L, 13] of the lists flat[off[l]:off[l+1]] (qf_qpp_raw)."""
    import torch
    dev = engine.require_device()
    flat = java_floats(flat)  # Gson's float of the JSON decimal (QPPBridge.java:67-70)
    nt, tf = textfeat.feature_arrays(texts)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    raw = engine.qpp_raw(t(flat) if flat.size else torch.zeros(1, dtype=torch.float64, device=dev),
                         t(off), 1, top_k, t(nt), t(tf))
    return raw.cpu().numpy()


class QPPBridge:
    """Same interface as the reference's Java bridge; the arithmetic runs on the GPU."""

    def __init__(self, java_dir: Optional[str] = None, persistent: bool = True):
        self.persistent = persistent
        self.qpp_method_names = list(config.qpp.methods)
        try:
            engine.require_device()
        except (RuntimeError, ImportError) as exc:  # the reference raises RuntimeError too
            raise RuntimeError(f"QPP engine unavailable: {exc}") from exc
        print("[QPP] MI355X QPP kernels ready", file=sys.stderr)

    def compute_batch(self, queries_scores: List[tuple]) -> List[QPPResult]:
        """[(query_text, scores)] -> one QPPResult per list, in input order."""
        if not queries_scores:
            return []
        texts = [str(q) for q, _ in queries_scores]
        lists = [list(s) for _, s in queries_scores]
        raw = _device_qpp(lists, texts)
        out = []
        for text, scores, row in zip(texts, lists, raw):
            vals = {} if len(scores) == 0 else dict(zip(QPP_METHODS, row.tolist()))
            out.append(QPPResult(query=text, retriever_name="batch", qpp_scores=vals,
                                 methods_used=self.qpp_method_names, processing_time_ms=0,
                                 predictions={}))
        return out

    def compute(self, query: str, scores: List[float], retriever_name: str = "unknown",
                methods: Optional[List[str]] = None) -> QPPResult:
        t0 = time.time()
        raw = _device_qpp([list(scores)], [query])[0]
        vals = {} if len(scores) == 0 else dict(zip(QPP_METHODS, raw.tolist()))
        return QPPResult(query=query, retriever_name=retriever_name, qpp_scores=vals,
                         methods_used=list(vals.keys()),
                         processing_time_ms=(time.time() - t0) * 1000, predictions={})


def _read_scores(res_path: str):
    """qid -> [scores] in file order, for lines with >= 5 fields (src/qpp.py:292-298):
    the reference's own loop, for the files the native reader leaves to it."""
    runs = defaultdict(list)
    with open(res_path, "r") as fh:
        for line in fh:
            f = line.strip().split()
            if len(f) >= 5:
                runs[f[0]].append(float(f[4]))
    return runs


def read_score_lists(res_path: str, top_k: int):
    """(qids, list_off, scores): every query's scores sorted descending and cut to
    top_k (src/qpp.py:292-305) — parsed and sorted natively (libqfio,
    qfio_read_score_lists); a file only Python reads exactly (non-ASCII bytes,
    digit underscores, NaN scores: include/qfio.h) goes through the reference's
    loop and sorted()."""
    from . import fastio
    got = fastio.read_score_lists(res_path, top_k)
    if got is not None:
        return got[:3]
    runs = _read_scores(res_path)
    qids = list(runs.keys())
    lists = [sorted(runs[q], reverse=True)[:top_k] for q in qids]
    off = np.zeros(len(qids) + 1, np.int64)
    np.cumsum([len(x) for x in lists], out=off[1:])
    flat = np.fromiter((x for s in lists for x in s), np.float64, count=int(off[-1]))
    return qids, off, flat


def compute_qpp_for_res_file(res_path: str, output_path: Optional[str] = None,
                             top_k: int = None, normalize: str = None,
                             queries_path: Optional[str] = None) -> Dict[str, List[float]]:
    """QPP of every query in a raw TREC .res file; writes <out>.qpp if asked
    (src/qpp.py:245-337).  Parse, per-query sort and top-k natively; the 13
    predictors (qf_qpp_raw) and the per-column normalisation on device."""
    top_k = top_k or config.processing.retrieval.top_k
    normalize = normalize or config.qpp.normalization
    if not os.path.exists(res_path):
        raise FileNotFoundError(f"Run file not found: {res_path}")
    texts = {}
    if queries_path and os.path.exists(queries_path):
        with open(queries_path, "r") as fh:
            for line in fh:
                q = json.loads(line)
                texts[q["_id"]] = q["text"]
    qids, off, flat = read_score_lists(res_path, top_k)
    if not qids:
        raise ValueError(f"No valid entries in run file: {res_path}")
    QPPBridge()
    raw = _device_qpp_flat(flat, off, [texts.get(q, q) for q in qids])
    empty = np.diff(off) == 0  # Java's empty map: every name 0.0 (src/qpp.py:321)
    if empty.any():
        raw[empty] = 0.0
    # columns in config.qpp.methods order, absent names 0.0 (src/qpp.py:319-322)
    names = list(config.qpp.methods)
    if names != QPP_METHODS:
        pos = {n: i for i, n in enumerate(QPP_METHODS)}
        cols = np.zeros((len(qids), len(names)))
        for j, m in enumerate(names):
            if m in pos:
                cols[:, j] = raw[:, pos[m]]
        raw = cols
    if normalize != "none":
        raw = _normalize_array(raw, normalize)
    results = {q: raw[i].tolist() for i, q in enumerate(qids)}
    if output_path:
        order = sorted(range(len(qids)), key=lambda i: int(qids[i]) if qids[i].isdigit() else qids[i])
        _write_qpp(output_path, [qids[i] for i in order], raw[order])
        print(f"Wrote QPP scores to {output_path}")
    return results


def _write_qpp(path: str, qids: List[str], vals: np.ndarray) -> None:
    """"{qid}\t" + "\t".join(f"{s:.6f}") per row (src/qpp.py:329-335)."""
    from . import fastio
    fmt = fastio.format_scores(np.ascontiguousarray(vals, np.float64).ravel())
    n = vals.shape[1] if vals.ndim == 2 else 0
    with open(path, "w") as fh:
        fh.write("".join(f"{q}\t" + "\t".join(fmt[i * n:(i + 1) * n]) + "\n"
                         for i, q in enumerate(qids)))


def _normalize_qpp(results: Dict[str, List[float]], method: str) -> Dict[str, List[float]]:
    """Per-column normalisation across queries (src/qpp.py:340-374), on device:
    minmax (min / max) or zscore (numpy's mean / population std, bit-exact)."""
    qids = list(results.keys())
    arr = np.asarray([results[q] for q in qids], dtype=np.float64).reshape(len(qids), -1)
    vals = _normalize_array(arr, method)
    return {q: [float(v) for v in vals[i]] for i, q in enumerate(qids)}


def _normalize_array(arr: np.ndarray, method: str) -> np.ndarray:
    """_normalize_qpp of a [Q, n_cols] array (rows = queries in results order)."""
    n_q, n_cols = arr.shape
    if n_cols > config.qpp.n_methods:  # method_values[i] of the reference (src/qpp.py:347-350)
        raise IndexError("list index out of range")
    if method == "minmax" and (n_cols < config.qpp.n_methods or not n_q):
        # the reference's minmax takes np.array([]).min() of every column no row
        # fills (config.qpp.methods shorter than n_methods, src/qpp.py:347-357)
        raise ValueError("zero-size array to reduction operation minimum which has no identity")
    # the kernels normalise 13 independent columns per row: pad to a multiple
    width = -(-max(n_cols, 1) // _lib.QPP_COLS) * _lib.QPP_COLS
    arr = np.ascontiguousarray(np.pad(arr, ((0, 0), (0, width - n_cols)))
                               .reshape(-1, _lib.QPP_COLS))
    rows_per = width // _lib.QPP_COLS
    method = "minmax" if method == "minmax" else "zscore"  # src/qpp.py:357-359: else -> zscore
    import torch
    dev = engine.require_device()
    raw = torch.from_numpy(arr).to(dev)
    # every list present; the padded row pieces of one query are the "retrievers"
    off = torch.arange(n_q * rows_per + 1, dtype=torch.int64, device=dev)
    stats = (engine.qpp_colminmax if method == "minmax" else engine.qpp_colmeanstd)(
        raw, off, rows_per)
    norm = engine.qpp_normalize(raw, stats, off, rows_per, method, qpp_index=0, want_norm=True,
                                want_micro=False, want_weights=False)["norm"]
    return norm.cpu().numpy().reshape(n_q, width)[:, :n_cols]

"""ctypes loader for oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"
_lib = None


def build() -> Path:
    srcs = [HERE / "fusion_oracle.c", HERE / "qpp_oracle.c", HERE / "eval_oracle.c",
            HERE / "synth_oracle.c"]
    if not LIB.exists() or any(s.stat().st_mtime > LIB.stat().st_mtime for s in srcs):
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        build()
        _lib = C.CDLL(str(LIB))
        vp, i64, i32 = C.c_void_p, C.c_int64, C.c_int32
        _lib.oracle_fuse.restype = C.c_int
        _lib.oracle_fuse.argtypes = [i64, i32, vp, vp, vp, vp, vp, i32, i32, vp, vp, vp, vp]
        _lib.oracle_minmax_per_query.restype = None
        _lib.oracle_minmax_per_query.argtypes = [vp, vp, i64, vp]
        _lib.oracle_eval.restype = C.c_int
        _lib.oracle_eval.argtypes = [i64, vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp]
        _lib.oracle_qpp_raw.restype = None
        _lib.oracle_qpp_raw.argtypes = [vp, vp, i64, vp, vp, vp, vp]
        _lib.oracle_synth_runs_nq.restype = C.c_int
        _lib.oracle_synth_runs_nq.argtypes = [i64, i64, i32, i32, C.c_uint64, vp, vp, i64, vp, vp,
                                              vp]
        _lib.oracle_det_log.restype = C.c_double
        _lib.oracle_det_log.argtypes = [C.c_double]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]


def fuse(list_off, docid, score, R, method, rrf_k=60, weights=None, rank=None):
    """Run the C oracle; returns (union_docid, union_count, perm, fused) numpy arrays."""
    list_off = np.ascontiguousarray(list_off, dtype=np.int64)
    docid = np.ascontiguousarray(docid, dtype=np.uint32)
    score = np.ascontiguousarray(score, dtype=np.float64)
    rank = None if rank is None else np.ascontiguousarray(rank, dtype=np.int32)
    weights = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
    E = int(list_off[-1]) if len(list_off) else 0
    Q = (len(list_off) - 1) // R
    ud = np.zeros(E, np.uint32)
    uc = np.zeros(Q, np.int32)
    perm = np.zeros(E, np.uint32)  # u may exceed 65,535 (qf_fuse_wide)
    fused = np.zeros(E, np.float64)
    m = METHODS.index(method) if isinstance(method, str) else int(method)
    rc = lib().oracle_fuse(Q, R, _p(list_off), _p(docid), _p(score), _p(rank), _p(weights), m,
                           rrf_k, _p(ud), _p(uc), _p(perm), _p(fused))
    if rc != 0:
        raise MemoryError("oracle_fuse failed")
    return ud, uc, perm, fused


def minmax_per_query(score, list_off):
    score = np.ascontiguousarray(score, dtype=np.float64)
    list_off = np.ascontiguousarray(list_off, dtype=np.int64)
    out = np.zeros_like(score)
    lib().oracle_minmax_per_query(_p(score), _p(list_off), len(list_off) - 1, _p(out))
    return out


def qpp_raw(score, list_off, num_terms, maxidf, avgidf):
    """13 raw predictors per list (lists already sorted desc / truncated)."""
    score = np.ascontiguousarray(score, dtype=np.float64)
    list_off = np.ascontiguousarray(list_off, dtype=np.int64)
    L = len(list_off) - 1
    nt = np.ascontiguousarray(np.broadcast_to(num_terms, (L,)), dtype=np.int32)
    mi = np.ascontiguousarray(np.broadcast_to(maxidf, (L,)), dtype=np.float64)
    ai = np.ascontiguousarray(np.broadcast_to(avgidf, (L,)), dtype=np.float64)
    out = np.zeros((L, 13), np.float64)
    lib().oracle_qpp_raw(_p(score), _p(list_off), L, _p(nt), _p(mi), _p(ai), _p(out))
    return out


EVAL_KINDS = {"ndcg": 0, "rr": 1, "r": 2, "p": 3, "ap": 4}


def _measure(name):
    import re
    m = re.fullmatch(r"([A-Za-z]+)(?:@(\d+))?", name)
    kind = EVAL_KINDS[m.group(1).lower()]
    return kind, int(m.group(2)) if m.group(2) else (0 if kind == 4 else 1 << 30)


def evaluate(off, docid, score, qrel_off, qrel_docid, qrel_rel, measures, text=False):
    """trec_eval restatement: [Q, len(measures)] float64 (NaN = not evaluated)."""
    off = np.ascontiguousarray(off, dtype=np.int64)
    docid = np.ascontiguousarray(docid, dtype=np.uint32)
    score = np.ascontiguousarray(score, dtype=np.float64)
    qrel_off = np.ascontiguousarray(qrel_off, dtype=np.int64)
    qrel_docid = np.ascontiguousarray(qrel_docid, dtype=np.uint32)
    qrel_rel = np.ascontiguousarray(qrel_rel, dtype=np.int32)
    spec = [_measure(m) for m in measures]
    kind = np.asarray([k for k, _ in spec], np.int32)
    cut = np.asarray([c for _, c in spec], np.int32)
    Q = len(off) - 1
    out = np.zeros((Q, len(spec)), np.float64)
    rc = lib().oracle_eval(Q, _p(off), _p(docid), _p(score), int(bool(text)), _p(qrel_off),
                           _p(qrel_docid), _p(qrel_rel), len(spec), _p(kind), _p(cut), _p(out))
    if rc != 0:
        raise MemoryError("oracle_eval")
    return out


def synth_runs_nq(q_begin, n_queries, R, K, seed, qrel_off, qrel_doc):
    """CPU regeneration of qf_synth_runs_nq (oracle/synth_oracle.c): list_off, docid,
    raw scores of lists [q_begin, q_begin + n_queries) x R, bit for bit."""
    qrel_off = np.ascontiguousarray(qrel_off, dtype=np.int64)
    qrel_doc = np.ascontiguousarray(qrel_doc, dtype=np.uint32)
    n = int(n_queries) * int(R)
    off = np.zeros(n + 1, np.int64)
    doc = np.zeros(n * int(K), np.uint32)
    sc = np.zeros(n * int(K), np.float64)
    rc = lib().oracle_synth_runs_nq(int(q_begin), int(n_queries), int(R), int(K), int(seed),
                                    _p(qrel_off), _p(qrel_doc), len(qrel_off) - 1, _p(off),
                                    _p(doc), _p(sc))
    if rc:
        raise MemoryError("oracle_synth_runs_nq")
    return off, doc, sc


def det_log(x: float) -> float:
    return float(lib().oracle_det_log(float(x)))

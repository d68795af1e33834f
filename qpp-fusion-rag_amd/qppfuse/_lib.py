"""ctypes binding of libqppfuse.so (C-ABI declared in include/qppfuse.h).

There is deliberately no fallback: if the HIP library is missing or fails to
load, every entry point of qppfuse raises.  See INTEGRATION.md.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

from ._build import LIB_PATH

QF_OK, QF_EINVAL, QF_ETOOBIG, QF_EHIP = 0, 1, 2, 3
QF_QSTATUS_TOOBIG, QF_QSTATUS_UNSORTED, QF_QSTATUS_RANKORDER, QF_QSTATUS_BADDOC, \
    QF_QSTATUS_DUPDOC = -1, -2, -3, -4, -5
QF_QSTATUS = {-1: "query exceeds the fusion kernel's entry limit",
              -2: "run list not sorted by score descending",
              -3: "rank column not non-decreasing within a run list",
              -4: "reserved docid 0xFFFFFFFF",
              -5: "a docno repeats within one run list (the host splits such lists)"}

COMBSUM, COMBMNZ, RRF, WCOMBSUM, WCOMBMNZ, WRRF, LEARNED, PROBFUSE, WRRF_MUL = \
    (1 << i for i in range(9))
METHOD_BITS = {"combsum": COMBSUM, "combmnz": COMBMNZ, "rrf": RRF,
               "wcombsum": WCOMBSUM, "wcombmnz": WCOMBMNZ, "wrrf": WRRF, "learned": LEARNED,
               "probfuse": PROBFUSE, "wrrf_mul": WRRF_MUL}
SCORE_F64, SCORE_MICRO = 0, 1
NORM_NONE, NORM_MINMAX, NORM_ZSCORE = 0, 1, 2
QPP_COLS = 13
MAX_RUNS = 32  # qf_fuse: retriever masks are 32-bit (include/qppfuse.h)
EVAL_NDCG, EVAL_RR, EVAL_R, EVAL_P, EVAL_AP = range(5)
EVAL_MAX_METRICS, EVAL_MAX_QRELS = 16, 256

# name -> (restype, argtypes); must match include/qppfuse.h (the *_wide entry points
# take the same arguments as their narrow forms: perm is a pointer either way)
_vp, _i32, _i64, _u64, _f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double
SIGNATURES = {
    "qf_version": (C.c_char_p, []),
    "qf_last_error": (C.c_char_p, []),
    "qf_max_entries_per_query": (C.c_int, []),
    "qf_max_entries_per_query_wide": (C.c_int, []),
    "qf_minmax_per_query": (C.c_int, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "qf_qpp_raw": (C.c_int, [_vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp]),
    "qf_qpp_colminmax": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "qf_minmax_colminmax": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    "qf_qpp_colmeanstd": (C.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "qf_qpp_normalize": (C.c_int, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    "qf_qpp_features": (C.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp]),
    "qf_fuse": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _i32,
                          _vp, _vp, _vp, _vp, _i64, _vp]),
    "qf_fuse_qpp": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32, _i32,
                              _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp]),
    "qf_fuse_qpp_micro": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i32, _i32,
                                    _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "qf_fuse_probfuse": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _vp,
                                   _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i64, _vp]),
    "qf_fused_topk": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp,
                                _vp]),
    "qf_eval": (C.c_int, [_i64, _vp, _i32, _vp, _vp, _vp, _vp, _i64, _i32, _i32, _vp, _vp, _vp,
                          _i32, _i32, _vp, _vp, _vp, _vp]),
    "qf_gbdt_predict": (C.c_int, [_i64, _vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _vp, _vp]),
    "qf_learned_weights": (C.c_int, [_i64, _vp, _i32, _i32, _vp, _vp, _vp]),
    "qf_learned_gbdt_weights": (C.c_int, [_i64, _vp, _vp, _vp, _vp, _i32, _i32, _vp, _i32, _i32,
                                          _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "qf_mlp_weights": (C.c_int, [_i64, _vp, _i32, _vp, _i32, _vp, _vp, _i32, _vp, _vp, _vp]),
    "qf_fuse_learned_f32": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, C.c_uint32, _i32,
                                      _vp, _vp, _vp, _vp, _i64, _vp]),
    "qf_synth_runs": (C.c_int, [_i64, _i64, _i32, _i32, _u64, _f64, _vp, _vp, _vp, _vp]),
    "qf_synth_runs_nq": (C.c_int, [_i64, _i64, _i32, _i32, _u64, _vp, _vp, _i64, _vp, _vp, _vp,
                                   _vp]),
    "qf_stream_copy": (C.c_int, [_vp, _vp, _i64, _vp]),
    "qf_fuse_workspace_bytes": (C.c_int64, [_i64, _i32, _i32, _i32, _i32]),
    "qf_fuse_ws": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _i32, _i32, _i32,
                             _vp, _vp, _vp, _i32, _vp, _i64, _vp, C.c_size_t, _vp]),
}
for _n in ("qf_fuse", "qf_fuse_probfuse", "qf_fuse_learned_f32", "qf_fused_topk"):
    SIGNATURES[_n + "_wide"] = SIGNATURES[_n]


class QPPFuseError(RuntimeError):
    """A libqppfuse call failed (maps the C status code and qf_last_error())."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"qppfuse error {code}: {msg}")
        self.code = code


_LIB = None


def lib() -> C.CDLL:
    """Load libqppfuse.so once; raise loudly when it is absent."""
    global _LIB
    if _LIB is None:
        import os
        path = Path(os.environ.get("QPPFUSE_LIB", LIB_PATH))  # dev override (variant builds)
        if not path.exists():
            raise ImportError(
                f"libqppfuse.so not built at {path}. Run `python __graft_entry__.py build` "
                "(hipcc --offload-arch=gfx950). qppfuse has no CPU fallback.")
        handle = C.CDLL(str(path))
        dev_build = "QPPFUSE_LIB" in os.environ  # an older build under A/B may lack new symbols
        for name, (res, args) in SIGNATURES.items():
            if dev_build and not hasattr(handle, name):
                continue
            fn = getattr(handle, name)
            fn.restype, fn.argtypes = res, args
        _LIB = handle
    return _LIB


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != QF_OK:
        msg = lib().qf_last_error().decode(errors="replace")
        if rc == QF_EINVAL:
            raise ValueError(f"{name}: {msg}")
        raise QPPFuseError(rc, f"{name}: {msg}")


def version() -> str:
    return lib().qf_version().decode()


def max_entries_per_query() -> int:
    return int(lib().qf_max_entries_per_query())


def max_entries_per_query_wide() -> int:
    return int(lib().qf_max_entries_per_query_wide())

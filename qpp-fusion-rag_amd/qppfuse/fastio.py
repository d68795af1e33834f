"""Native TREC run I/O (libqfio.so, csrc/qf_io.cpp) for the fusion path.

load_runs parses every run file in C++ (memory-mapped, multithreaded) straight
into the packed RunSet the device kernels read, and also returns the
DataFrames the reference's load_runs returns (src/fusion.py:46-76) — qid /
docno / iter / runid as object columns of the interned strings, rank
int64, score float64, rows in file order — with the RunSet cached for them, so
the fusions that follow skip packing.  write_run writes one fused run the way
write_runfile does (src/fusion.py:480-492), formatting in C++ with Python's
exact "%.6f".
"""
from __future__ import annotations

import ctypes as C
import collections
import os
from pathlib import Path
from typing import Dict, List, Sequence, Tuple

import numpy as np
import pandas as pd

from ._build import IO_LIB_PATH

_LIB = None
_vp, _i32, _i64 = C.c_void_p, C.c_int32, C.c_int64


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = Path(os.environ.get("QPPFUSE_IO_LIB", IO_LIB_PATH))
        if not path.exists():
            raise ImportError(f"{path} is missing: build it with `python __graft_entry__.py build`")
        L = C.CDLL(str(path))
        L.qfio_last_error.restype = C.c_char_p
        L.qfio_load_runs.restype = C.c_int
        L.qfio_load_runs.argtypes = [C.POINTER(C.c_char_p), _i32, _i32, C.POINTER(_vp)]
        L.qfio_runset_sizes.restype = None
        L.qfio_runset_sizes.argtypes = [_vp, _vp]
        L.qfio_runset_csr.restype = C.c_int
        L.qfio_runset_csr.argtypes = [_vp] + [_vp] * 5
        L.qfio_runset_strings.restype = C.c_int
        L.qfio_runset_strings.argtypes = [_vp] + [_vp] * 8
        L.qfio_runset_rows.restype = C.c_int
        L.qfio_runset_rows.argtypes = [_vp] + [_vp] * 7
        L.qfio_join_lines.restype = C.c_int
        L.qfio_join_lines.argtypes = [_vp, _vp, _i64, _vp]
        L.qfio_gather_strings.restype = _i64
        L.qfio_gather_strings.argtypes = [_vp, _vp, _vp, _i64, _vp, _vp]
        L.qfio_gather_chars.restype = C.c_int
        L.qfio_gather_chars.argtypes = [_vp, _vp, _vp, _i64, _vp, _vp]
        L.qfio_repeat_offsets.restype = None
        L.qfio_repeat_offsets.argtypes = [_i64, _i64, _vp]
        L.qfio_hash_bytes.restype = C.c_uint64
        L.qfio_hash_bytes.argtypes = [_vp, _i64]
        L.qfio_runset_drop_text.restype = None
        L.qfio_runset_drop_text.argtypes = [_vp]
        L.qfio_runset_views.restype = None
        L.qfio_runset_views.argtypes = [_vp, _vp]
        L.qfio_runset_free.restype = None
        L.qfio_runset_free.argtypes = [_vp]
        L.qfio_format_score.restype = C.c_size_t
        L.qfio_format_score.argtypes = [C.c_double, C.c_char_p]
        L.qfio_read_score_lists.restype = C.c_int
        L.qfio_read_score_lists.argtypes = [C.c_char_p, _i32, _i32, C.POINTER(_vp)]
        L.qfio_scorelists_sizes.restype = None
        L.qfio_scorelists_sizes.argtypes = [_vp, _vp]
        L.qfio_scorelists_get.restype = C.c_int
        L.qfio_scorelists_get.argtypes = [_vp] * 5
        L.qfio_scorelists_free.restype = None
        L.qfio_scorelists_free.argtypes = [_vp]
        for fn in (L.qfio_write_run, L.qfio_write_run32):
            fn.restype = C.c_int
            fn.argtypes = [C.c_char_p, _i64] + [_vp] * 10 + [C.c_char_p, _i32]
        _LIB = L
    return _LIB


def _check(rc: int, what: str):
    if rc == 0:
        return
    msg = lib().qfio_last_error().decode(errors="replace")
    if rc == 2:
        raise FileNotFoundError(msg)
    if rc == 4:
        raise ValueError(f"{what}: {msg}")
    raise OSError(f"{what}: {msg}")


class _RunSetOwner:
    """A parsed qfio_runset whose column buffers back numpy arrays: freed when
    the last array made by array() (each holds a reference) is collected."""

    def __init__(self, h):
        self.h = h

    def array(self, ptr, n: int, dtype) -> np.ndarray:
        dt = np.dtype(dtype)
        if n == 0 or not ptr:
            return np.zeros(n, dt)
        buf = (C.c_char * (n * dt.itemsize)).from_address(ptr)
        buf._owner = self  # the ctypes buffer is the array's base
        return np.frombuffer(buf, dt, n)

    def __del__(self):
        if self.h is not None and _LIB is not None:
            _LIB.qfio_runset_free(self.h)
            self.h = None


def _p(a: np.ndarray):
    return a.ctypes.data_as(_vp)


def read_score_lists(path: str, top_k: int, n_threads: int = 0):
    """compute_qpp_for_res_file's read of a raw run (src/qpp.py:292-305), natively
    (qfio_read_score_lists): (qids in first-appearance order, list_off[Q+1], the
    descending-sorted [:top_k] scores of every query, rows read).  None when the
    file needs the reference's own Python reading (include/qfio.h QFIO_EPYTHON)."""
    L = lib()
    h = _vp()
    rc = L.qfio_read_score_lists(path.encode(), int(top_k), n_threads, C.byref(h))
    if rc == 5:
        return None
    if rc == 4:  # float()'s own ValueError text
        raise ValueError(L.qfio_last_error().decode(errors="replace"))
    _check(rc, "read_score_lists")
    try:
        sz = np.zeros(4, np.int64)
        L.qfio_scorelists_sizes(h, _p(sz))
        Q, n, qb, rows = (int(x) for x in sz)
        qoff = np.empty(Q + 1, np.int64)
        qch = np.empty(max(qb, 1), np.uint8)
        loff = np.empty(Q + 1, np.int64)
        sc = np.empty(max(n, 1), np.float64)
        _check(L.qfio_scorelists_get(h, _p(qoff), _p(qch), _p(loff), _p(sc)), "read_score_lists")
    finally:
        L.qfio_scorelists_free(h)
    raw = qch[:qb].tobytes()
    qids = [raw[qoff[i]:qoff[i + 1]].decode() for i in range(Q)]  # ASCII (else EPYTHON)
    return qids, loff, sc[:n], rows


def _strings(off: np.ndarray, chars: np.ndarray) -> np.ndarray:
    """Offsets + bytes -> object array of str (C join with newlines, one decode + split)."""
    n = len(off) - 1
    if n == 0:
        return np.zeros(0, dtype=object)
    blob = np.empty(int(off[-1]) + n, np.uint8)
    _check(lib().qfio_join_lines(_p(np.ascontiguousarray(off, np.int64)), _p(chars), n, _p(blob)),
           "join_lines")
    out = np.empty(n, dtype=object)
    out[:] = blob.tobytes().decode().split("\n")[:n]
    return out


def arrow_strings(off: np.ndarray, chars: np.ndarray, codes: np.ndarray):
    """Per-row strings (codes into the table off/chars) as a pandas ArrowStringArray:
    the bytes gathered in C++ straight into Arrow string buffers, no Python str
    per row (they are made when an element is read).  A column of one value
    (iter "Q0", a run's tag) is a repeat."""
    import pyarrow as pa
    codes = np.ascontiguousarray(codes, np.uint32)
    n = len(codes)
    L = lib()
    out_off = np.empty(n + 1, np.int64)
    if n and codes[0] == codes[-1] and (codes == codes[0]).all():
        v = bytes(chars[off[codes[0]]:off[codes[0] + 1]])
        L.qfio_repeat_offsets(len(v), n, _p(out_off))
        arr = pa.LargeStringArray.from_buffers(n, pa.py_buffer(out_off), pa.py_buffer(v * n))
        return pd.arrays.ArrowStringArray(pa.chunked_array([arr]))
    # large_string (int64 offsets): what pandas' ArrowStringArray holds, so no cast
    nb = L.qfio_gather_strings(_p(off), _p(chars), _p(codes), n, _p(out_off), None)
    if nb < 0:
        raise ValueError("gather_strings: bad arguments")
    buf = np.empty(max(int(nb), 1), np.uint8)
    if L.qfio_gather_chars(_p(off), _p(chars), _p(codes), n, _p(out_off), _p(buf)) != 0:
        raise ValueError("gather_chars: bad arguments")
    arr = pa.LargeStringArray.from_buffers(n, pa.py_buffer(out_off), pa.py_buffer(buf[:nb]))
    return pd.arrays.ArrowStringArray(pa.chunked_array([arr]))


def frame_strings() -> str:
    """String columns of the frames load_runs returns: "arrow" (default; pandas'
    string[pyarrow], the dtype pandas >= 3 gives read_csv text by default) or
    "object" (Python str objects, pandas 2's read_csv dtype); QPPFUSE_FRAME_STRINGS."""
    v = os.environ.get("QPPFUSE_FRAME_STRINGS", "arrow")
    if v not in ("arrow", "object"):
        raise ValueError(f"QPPFUSE_FRAME_STRINGS must be 'arrow' or 'object', not {v!r}")
    return v


def hash_bytes(a: np.ndarray) -> int:
    """64-bit content digest of a contiguous array (qfio_hash_bytes, multi-threaded)."""
    a = np.ascontiguousarray(a)
    return int(lib().qfio_hash_bytes(_p(a) if a.size else None, a.nbytes))


def format_score(x: float) -> str:
    buf = C.create_string_buffer(400)
    n = lib().qfio_format_score(float(x), buf)
    return buf.raw[:n].decode()


def format_scores(x: np.ndarray) -> List[str]:
    """[f"{v:.6f}" for v in x] (the .qpp writer's format, src/qpp.py:333)."""
    return [f"{v:.6f}" for v in np.asarray(x, np.float64).tolist()]


def parse_runs(paths: Sequence[str], names: Sequence[str], n_threads: int = 0):
    """Parse run files -> (RunSet, {name: DataFrame})."""
    from .runset import RunSet
    L = lib()
    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    h = _vp()
    _check(L.qfio_load_runs(arr, len(paths), int(n_threads), C.byref(h)), "load_runs")
    try:
        sz = np.zeros(8, np.int64)
        L.qfio_runset_sizes(h, _p(sz))
        Q, D, E, qb, db, flags = (int(x) for x in sz[:6])
        micro_ok = flags & 1
        n_iter, n_tag = int(sz[6]) & 0xFFFFFFFF, int(sz[6]) >> 32
        ib, tb = int(sz[7]) & 0xFFFFFFFF, int(sz[7]) >> 32
        R = len(paths)
        # (every offset and byte is written by qfio_runset_strings)
        qo, qc = np.empty(Q + 1, np.int64), np.zeros(max(qb, 1), np.uint8)
        do, dc = np.empty(D + 1, np.int64), np.empty(max(db, 1), np.uint8)
        io, ic = np.empty(n_iter + 1, np.int64), np.zeros(max(ib, 1), np.uint8)
        to, tc = np.empty(n_tag + 1, np.int64), np.zeros(max(tb, 1), np.uint8)
        L.qfio_runset_strings(h, _p(qo), _p(qc), _p(do), _p(dc), _p(io), _p(ic), _p(to), _p(tc))
        # the columns stay in the run set's buffers (no copies): numpy views that
        # keep the run set alive until the last of them is gone
        L.qfio_runset_drop_text(h)  # the text is copied out; unmap the files
        owner = _RunSetOwner(h)
        h = None
        ptrs = (C.c_void_p * 12)()
        L.qfio_runset_views(owner.h, ptrs)
        view = lambda i, n, dt: owner.array(ptrs[i], n, dt)
        list_off = view(0, Q * R + 1, np.int64)
        docid, score = view(1, E, np.uint32), view(2, E, np.float64)
        micro = view(3, E, np.int32) if micro_ok else None
        rank = view(4, E, np.int64)
        fo = view(5, R + 1, np.int64)
        rq, rd = view(6, E, np.uint32), view(7, E, np.uint32)
        ri, rt = view(8, E, np.uint32), view(9, E, np.uint32)
        rr, rsc = view(10, E, np.int64), view(11, E, np.float64)
    finally:
        if h is not None:
            L.qfio_runset_free(h)
    from .runset import StringTable
    qids = _strings(qo, qc)
    dcb = dc.tobytes()
    rs = RunSet(qids=list(qids), rankers=list(names), docnos=StringTable(do, dcb),
                list_off=list_off, docid=docid, score=score, rank=rank, micro=micro)
    rs.rank_is_position = bool(flags & 2)
    rs.canonical = bool(flags & 4)
    rs.has_dups = bool(flags & 8)
    rs._strtab = {"qid": (qo, qc.tobytes()), "docno": (do, dcb)}
    frames = {}
    if frame_strings() == "arrow":
        for r, name in enumerate(names):
            a, b = int(fo[r]), int(fo[r + 1])
            frames[name] = pd.DataFrame({
                "qid": arrow_strings(qo, qc, rq[a:b]), "iter": arrow_strings(io, ic, ri[a:b]),
                "docno": arrow_strings(do, dc, rd[a:b]), "rank": rr[a:b], "score": rsc[a:b],
                "runid": arrow_strings(to, tc, rt[a:b])}, copy=False)
        return rs, frames
    docnos = rs.docnos.materialize()
    iters, tags = _strings(io, ic), _strings(to, tc)

    def column(strings, codes):
        # a column of one value (the usual iter "Q0" / a file's tag) is a broadcast
        if len(codes) and codes[0] == codes[-1] and (codes == codes[0]).all():
            return np.full(len(codes), strings[codes[0]], dtype=object)
        return strings[codes]

    for r, name in enumerate(names):
        a, b = int(fo[r]), int(fo[r + 1])
        frames[name] = pd.DataFrame({
            "qid": qids[rq[a:b]], "iter": column(iters, ri[a:b]), "docno": docnos[rd[a:b]],
            "rank": rr[a:b], "score": rsc[a:b], "runid": column(tags, rt[a:b])}, copy=False)
    return rs, frames


class DocnoTable:
    """The docno table of the last read_run_rows call: the object array of str it
    returned with the UTF-8 offsets / bytes it was decoded from.  The evaluator
    (evaluation._run_arrays_flat) codes rows that hold these very str objects by
    identity — no hashing or sorting of millions of Python strings — and sorts the
    table once in Arrow (byte order of UTF-8 = code-point order, Python's order)."""

    def __init__(self, objs: np.ndarray, off: np.ndarray, chars: np.ndarray):
        self.objs, self.off, self.chars = objs, off, chars
        self._ids = self._sorted = None

    def id_index(self) -> pd.Index:
        """pandas Index of every element's id() (a hash table: position by identity)."""
        if self._ids is None:
            self._ids = pd.Index(np.fromiter(map(id, self.objs), np.uint64, len(self.objs)))
        return self._ids

    def sorted_order(self) -> np.ndarray:
        """Element positions in ascending string order."""
        if self._sorted is None:
            import pyarrow as pa
            import pyarrow.compute as pc
            arr = pa.LargeStringArray.from_buffers(
                len(self.objs), pa.py_buffer(np.ascontiguousarray(self.off, np.int64)),
                pa.py_buffer(np.ascontiguousarray(self.chars, np.uint8)))
            self._sorted = pc.sort_indices(arr).to_numpy().astype(np.int64)
        return self._sorted


# the last table only (a run being evaluated is the one just loaded): bounded memory
docno_tables: "collections.deque[DocnoTable]" = collections.deque(maxlen=1)


def read_run_rows(path: str, n_threads: int = 0):
    """One TREC run file's rows in file order: (qids, docnos, qid code, docno code,
    rank, score) — the string tables as object arrays, the codes into them, rank
    int64 and score float64 as parsed by qfio (the loader of load_runs).  Raises
    ValueError for a file the loader rejects (a line without exactly 6 fields),
    FileNotFoundError for a missing one."""
    L = lib()
    arr = (C.c_char_p * 1)(os.fsencode(path))
    h = _vp()
    _check(L.qfio_load_runs(arr, 1, int(n_threads), C.byref(h)), "read_run_rows")
    try:
        sz = np.zeros(8, np.int64)
        L.qfio_runset_sizes(h, _p(sz))
        Q, D, E, qb, db = (int(x) for x in sz[:5])
        n_iter, n_tag = int(sz[6]) & 0xFFFFFFFF, int(sz[6]) >> 32
        ib, tb = int(sz[7]) & 0xFFFFFFFF, int(sz[7]) >> 32
        qo, qc = np.empty(Q + 1, np.int64), np.zeros(max(qb, 1), np.uint8)
        do, dc = np.empty(D + 1, np.int64), np.empty(max(db, 1), np.uint8)
        io, ic = np.empty(n_iter + 1, np.int64), np.zeros(max(ib, 1), np.uint8)
        to, tc = np.empty(n_tag + 1, np.int64), np.zeros(max(tb, 1), np.uint8)
        L.qfio_runset_strings(h, _p(qo), _p(qc), _p(do), _p(dc), _p(io), _p(ic), _p(to), _p(tc))
        L.qfio_runset_drop_text(h)
        owner = _RunSetOwner(h)
        h = None
        ptrs = (C.c_void_p * 12)()
        L.qfio_runset_views(owner.h, ptrs)
        rq, rd = owner.array(ptrs[6], E, np.uint32), owner.array(ptrs[7], E, np.uint32)
        rr, rsc = owner.array(ptrs[10], E, np.int64), owner.array(ptrs[11], E, np.float64)
    finally:
        if h is not None:
            L.qfio_runset_free(h)
    docnos = _strings(do, dc)
    docno_tables.append(DocnoTable(docnos, do, dc))
    return _strings(qo, qc), docnos, rq, rd, rr, rsc


def string_table(rs, which: str) -> Tuple[np.ndarray, bytes]:
    """(offsets [n+1], bytes) of a RunSet's qids or docnos (cached)."""
    tab = getattr(rs, "_strtab", None)
    if tab is None:
        tab = rs._strtab = {}
    if which not in tab:
        vals = rs.qids if which == "qid" else rs.docnos
        enc = [str(v).encode() for v in vals]
        off = np.zeros(len(enc) + 1, np.int64)
        np.cumsum([len(e) for e in enc], out=off[1:])
        tab[which] = (off, b"".join(enc))
    return tab[which]


def write_run(path: str, order: np.ndarray, qbase: np.ndarray, counts: np.ndarray,
              union_docid: np.ndarray, perm: np.ndarray, fused: np.ndarray, rs, tag: str,
              n_threads: int = 0, qid_table=None) -> None:
    """One fused run -> TREC text (queries in `order`, documents as ranked)."""
    qo, qc = string_table(rs, "qid") if qid_table is None else qid_table
    do, dc = string_table(rs, "docno")
    order = np.ascontiguousarray(order, np.int64)
    qbase = np.ascontiguousarray(qbase, np.int64)
    counts = np.ascontiguousarray(counts, np.int32)
    ud = np.ascontiguousarray(union_docid, np.uint32)
    wide = np.asarray(perm).dtype == np.uint32  # qf_fuse_wide's perm
    pm = np.ascontiguousarray(perm, np.uint32 if wide else np.uint16)
    fz = np.ascontiguousarray(fused, np.float64)
    qcb = np.frombuffer(qc, np.uint8) if qc else np.zeros(1, np.uint8)
    dcb = np.frombuffer(dc, np.uint8) if dc else np.zeros(1, np.uint8)
    fn = lib().qfio_write_run32 if wide else lib().qfio_write_run
    _check(fn(os.fsencode(path), len(order), _p(order), _p(qbase), _p(counts),
                                _p(ud), _p(pm), _p(fz), _p(qo), _p(qcb), _p(do), _p(dcb),
                                tag.encode(), int(n_threads)), "write_runfile")

"""Host-side packing of run lists into the CSR layout the HIP kernels read.

Layout (query-major, see include/qppfuse.h): Q queries in sorted-qid order (the
order the reference's weighted loops visit, src/fusion.py:264), R rankers in
`runs` dict order (os.listdir order from load_runs, src/fusion.py:60), list
(q, r) = entries [list_off[q*R + r], list_off[q*R + r + 1]) in file row order.
docnos are interned to uint32 ids (0xFFFFFFFF reserved); scores are sent as
int32 micro-units whenever every value is exactly a 6-decimal number (true for
every .norm.res file, which is "%.6f" text), else as float64.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import pandas as pd


class StringTable:
    """docid -> docno over the native parser's (offsets, bytes) table, in docno
    order: Python str objects are made only for what is looked up (a few
    thousand per query), and the whole object array only when one is asked for
    (np.asarray, searchsorted) — load_runs no longer builds ~10^7 of them."""

    _SMALL = 65536  # lookups up to this size decode the bytes directly

    def __init__(self, off: np.ndarray, chars: bytes):
        self.off = off
        self.chars = chars
        self._all: Optional[np.ndarray] = None

    def __len__(self) -> int:
        return len(self.off) - 1

    def materialize(self) -> np.ndarray:
        if self._all is None:
            from .fastio import _strings
            self._all = _strings(self.off, np.frombuffer(self.chars, np.uint8)
                                 if self.chars else np.zeros(1, np.uint8))
        return self._all

    def __iter__(self):
        return iter(self.materialize())

    def __array__(self, dtype=None, copy=None):
        a = self.materialize()
        return a if dtype is None else a.astype(dtype)

    def __getitem__(self, idx):
        if self._all is not None:
            return self._all[idx]
        if isinstance(idx, (int, np.integer)):
            i = int(idx)
            if not -len(self) <= i < len(self):
                raise IndexError(f"docid {i} out of range for {len(self)} docnos")
            i %= len(self)
            return self.chars[self.off[i]:self.off[i + 1]].decode()
        if isinstance(idx, slice):
            return self.materialize()[idx]
        idx = np.asarray(idx)
        if idx.dtype == bool or idx.size > self._SMALL:
            return self.materialize()[idx]
        o, c = self.off, self.chars
        out = np.empty(idx.shape, dtype=object)
        flat = out.reshape(-1)
        for k, i in enumerate(idx.reshape(-1).tolist()):
            flat[k] = c[o[i]:o[i + 1]].decode()
        return out


@dataclass
class RunSet:
    qids: List[str]
    rankers: List[str]
    docnos: object                # docid -> docno: object array or StringTable
    list_off: np.ndarray          # int64 [Q*R + 1]
    docid: np.ndarray             # uint32 [E]
    score: np.ndarray             # float64 [E]
    rank: np.ndarray              # int64 [E] (file rank column)
    micro: Optional[np.ndarray] = None   # int32 [E] when exact
    rank_is_position: bool = True        # rank == position + 1 in every list
    canonical: bool = True               # file order == score-desc order == rank order
    has_dups: bool = False               # a docno repeats inside one list
    base_ranker: Optional[np.ndarray] = None  # expand_duplicates: ranker of each virtual run
    _device: Dict[str, object] = field(default_factory=dict, repr=False)

    @property
    def n_queries(self) -> int:
        return len(self.qids)

    @property
    def n_rankers(self) -> int:
        return len(self.rankers)

    @property
    def n_entries(self) -> int:
        return int(self.list_off[-1])

    def max_entries(self) -> int:
        R = self.n_rankers
        qo = self.list_off[::R]
        return int(np.max(np.diff(qo))) if len(qo) > 1 else 0

    def query_base(self) -> np.ndarray:
        return self.list_off[:-1:self.n_rankers] if self.n_queries else np.zeros(0, np.int64)

    def to_device(self, device=None):
        """Upload once (cached); returns dict of torch tensors."""
        import torch
        if self._device:
            return self._device
        dev = device or torch.device("cuda")
        d = {"list_off": torch.from_numpy(self.list_off).to(dev),
             "docid": torch.from_numpy(self.docid.view(np.int32)).to(dev)}
        if self.micro is not None:
            d["score"] = torch.from_numpy(self.micro).to(dev)
        else:
            d["score"] = torch.from_numpy(self.score).to(dev)
        d["rank"] = (None if self.rank_is_position
                     else torch.from_numpy(self.rank.astype(np.int32)).to(dev))
        self._device = d
        return d


def _micro_encoding(score: np.ndarray) -> Optional[np.ndarray]:
    if score.size == 0:
        return np.zeros(0, np.int32)
    if not np.all(np.isfinite(score)):
        return None
    m = np.rint(score * 1e6)
    if np.any(np.abs(m) >= 2**31 - 1):
        return None
    if not np.array_equal(m / 1e6, score) or np.any((score == 0) & np.signbit(score)):
        return None  # a -0.0 score is not the micro-unit 0
    return m.astype(np.int32)


def pack_frames(runs: Dict[str, pd.DataFrame]) -> RunSet:
    """Pack the reference's {ranker: DataFrame[qid, docno, rank, score, ...]}."""
    if not runs:
        raise ValueError("no runs to fuse")
    rankers = list(runs.keys())
    R = len(rankers)
    qid_parts, doc_parts, score_parts, rank_parts, r_parts = [], [], [], [], []
    for r, name in enumerate(rankers):
        df = runs[name]
        qid_parts.append(df["qid"].astype(str).to_numpy())
        doc_parts.append(df["docno"].astype(str).to_numpy())
        score_parts.append(df["score"].to_numpy(dtype=np.float64))
        rank_parts.append(df["rank"].to_numpy(dtype=np.int64))
        r_parts.append(np.full(len(df), r, dtype=np.int64))
    qid_all = np.concatenate(qid_parts)
    doc_all = np.concatenate(doc_parts)
    score_all = np.concatenate(score_parts)
    rank_all = np.concatenate(rank_parts)
    r_all = np.concatenate(r_parts)
    qids = sorted(set(qid_all.tolist()))
    qcode = pd.Categorical(qid_all, categories=qids).codes.astype(np.int64)
    # ids in docno string order: trec_eval breaks score ties by docno (qf_eval)
    dcode, docnos = pd.factorize(doc_all, sort=True)
    if len(docnos) >= 0xFFFFFFFF:
        raise ValueError("too many distinct docnos for uint32 ids")
    key = qcode * R + r_all
    order = np.argsort(key, kind="stable")
    key_s = key[order]
    Q = len(qids)
    counts = np.bincount(key_s, minlength=Q * R)
    list_off = np.zeros(Q * R + 1, dtype=np.int64)
    np.cumsum(counts, out=list_off[1:])
    docid = dcode[order].astype(np.uint32)
    score = score_all[order]
    rank = rank_all[order]
    rs = RunSet(qids=qids, rankers=rankers, docnos=np.asarray(docnos, dtype=object),
                list_off=list_off, docid=docid, score=score, rank=rank)
    _analyse(rs, key_s)
    return rs


def _analyse(rs: RunSet, key_s: np.ndarray) -> None:
    """Order / uniqueness properties the kernels rely on (include/qppfuse.h)."""
    E = rs.n_entries
    same = key_s[1:] == key_s[:-1] if E > 1 else np.zeros(0, bool)
    # duplicates of a docno inside one list (handled by dedupe_keep_last /
    # expand_duplicates, the reference's two behaviours)
    if E > 1:
        o = np.lexsort((rs.docid, key_s))
        dup = (key_s[o][1:] == key_s[o][:-1]) & (rs.docid[o][1:] == rs.docid[o][:-1])
        rs.has_dups = bool(dup.any())
    score_ok = bool(np.all(rs.score[1:][same] <= rs.score[:-1][same])) if E > 1 else True
    rank_inc = bool(np.all(rs.rank[1:][same] > rs.rank[:-1][same])) if E > 1 else True
    pos = np.arange(E, dtype=np.int64) - np.repeat(rs.list_off[:-1], np.diff(rs.list_off))
    rs.rank_is_position = bool(np.array_equal(rs.rank, pos + 1))
    rs.canonical = score_ok and rank_inc
    rs.micro = _micro_encoding(rs.score)


def reorder(rs: RunSet, by: str) -> RunSet:
    """A copy whose lists are ordered by score (desc, stable) or rank (asc)."""
    E = rs.n_entries
    lid = np.repeat(np.arange(len(rs.list_off) - 1), np.diff(rs.list_off))
    if by == "score":
        o = np.lexsort((np.arange(E), -rs.score, lid))
    elif by == "rank":
        o = np.lexsort((np.arange(E), rs.rank, lid))
    else:
        raise ValueError(by)
    out = RunSet(qids=rs.qids, rankers=rs.rankers, docnos=rs.docnos, list_off=rs.list_off,
                 docid=rs.docid[o], score=rs.score[o], rank=rs.rank[o],
                 base_ranker=rs.base_ranker)
    _share_strings(rs, out)
    _analyse(out, lid[o])
    if by == "rank":
        # the kernel's order check is on scores; rank order is what W-RRF needs
        out.canonical = True
    return out


def _share_strings(src: RunSet, dst: RunSet) -> None:
    tab = getattr(src, "_strtab", None)
    if tab is not None:
        dst._strtab = tab


def _list_ids(rs: RunSet) -> np.ndarray:
    return np.repeat(np.arange(len(rs.list_off) - 1), np.diff(rs.list_off))


def _occurrence(lid: np.ndarray, docid: np.ndarray) -> np.ndarray:
    """For every entry: how many earlier entries of its list hold the same docno."""
    E = len(lid)
    o = np.lexsort((np.arange(E), docid, lid))
    same = np.zeros(E, bool)
    if E > 1:
        same[1:] = (lid[o][1:] == lid[o][:-1]) & (docid[o][1:] == docid[o][:-1])
    # run-length position inside each group of equal (list, docno)
    idx = np.arange(E)
    start = np.where(same, 0, idx)
    np.maximum.accumulate(start, out=start)
    occ = np.empty(E, np.int64)
    occ[o] = idx - start
    return occ


def dedupe_keep_last(rs: RunSet) -> RunSet:
    """One entry per docno per list, at its FIRST position with its LAST score.

    What the ranx methods see: _df_runs_to_ranx builds {qid: {docno: score}} row
    by row (src/fusion.py:459-464), and a repeated dict key keeps its insertion
    position while taking the new value.  The rank column keeps the first row's."""
    if not rs.has_dups:
        return rs
    lid = _list_ids(rs)
    E = rs.n_entries
    occ = _occurrence(lid, rs.docid)
    # entries grouped by (list, docno), positions ascending inside a group; the
    # group's last entry's score is broadcast to the group
    o = np.lexsort((np.arange(E), rs.docid, lid))
    gid = np.zeros(E, np.int64)
    if E > 1:
        gid[1:] = np.cumsum(~((lid[o][1:] == lid[o][:-1]) & (rs.docid[o][1:] == rs.docid[o][:-1])))
    last_idx = np.zeros(gid[-1] + 1 if E else 0, np.int64)
    last_idx[gid] = o  # o is position-ascending inside a group: the last write wins
    score = rs.score.copy()
    score[o] = rs.score[last_idx[gid]]
    keep = occ == 0
    counts = np.bincount(lid[keep], minlength=len(rs.list_off) - 1)
    list_off = np.zeros(len(rs.list_off), np.int64)
    np.cumsum(counts, out=list_off[1:])
    out = RunSet(qids=rs.qids, rankers=rs.rankers, docnos=rs.docnos, list_off=list_off,
                 docid=rs.docid[keep], score=score[keep], rank=rs.rank[keep])
    _share_strings(rs, out)
    _analyse(out, lid[keep])
    return out


def expand_duplicates(rs: RunSet) -> RunSet:
    """Every repeated row of a list moved to a virtual run right after its ranker.

    What the weighted loops and learned fusion's groupby do with a docno that
    repeats inside one list: every row adds its own contribution, rows in file
    order (src/fusion.py:273-277, 321-324, 372-374, 440-441).  The k-th
    occurrence (k >= 1) of a docno in ranker r goes to virtual run (r, k), placed
    after (r, k-1): a document's contributions are then summed in retriever
    order exactly as the reference adds its rows, and its first occurrence — in
    run (r, 0) — still fixes the first-seen order.  Virtual runs take their
    ranker's weight (base_ranker) and carry the file rank column."""
    if not rs.has_dups:
        return rs
    R = rs.n_rankers
    Q = rs.n_queries
    lid = _list_ids(rs)
    occ = _occurrence(lid, rs.docid)
    q, r = np.divmod(lid, R)
    kmax = np.zeros(R, np.int64)
    np.maximum.at(kmax, r, occ)
    first = np.zeros(R + 1, np.int64)  # virtual run index of (r, 0)
    np.cumsum(kmax + 1, out=first[1:])
    R2 = int(first[-1])
    vr = first[r] + occ
    key = q * R2 + vr
    o = np.lexsort((np.arange(len(key)), key))
    counts = np.bincount(key, minlength=Q * R2)
    list_off = np.zeros(Q * R2 + 1, np.int64)
    np.cumsum(counts, out=list_off[1:])
    base = np.repeat(np.arange(R), kmax + 1)
    names = [rs.rankers[b] if k == 0 else f"{rs.rankers[b]}#dup{k}"
             for b, k in zip(base, np.concatenate([np.arange(k + 1) for k in kmax]))]
    out = RunSet(qids=rs.qids, rankers=names, docnos=rs.docnos, list_off=list_off,
                 docid=rs.docid[o], score=rs.score[o], rank=rs.rank[o],
                 base_ranker=base if rs.base_ranker is None else rs.base_ranker[base])
    _share_strings(rs, out)
    _analyse(out, key[o])
    out.rank_is_position = False  # positions inside a virtual run are not file ranks
    return out

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


@dataclass
class RunSet:
    qids: List[str]
    rankers: List[str]
    docnos: np.ndarray            # object array: docid -> docno
    list_off: np.ndarray          # int64 [Q*R + 1]
    docid: np.ndarray             # uint32 [E]
    score: np.ndarray             # float64 [E]
    rank: np.ndarray              # int64 [E] (file rank column)
    micro: Optional[np.ndarray] = None   # int32 [E] when exact
    rank_is_position: bool = True        # rank == position + 1 in every list
    canonical: bool = True               # file order == score-desc order == rank order
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
    # duplicates of a docno inside one list
    if E > 1:
        o = np.lexsort((rs.docid, key_s))
        dup = (key_s[o][1:] == key_s[o][:-1]) & (rs.docid[o][1:] == rs.docid[o][:-1])
        if dup.any():
            i = int(o[1:][dup][0])
            q, r = divmod(int(key_s[i]), rs.n_rankers)
            raise ValueError(
                f"docno '{rs.docnos[rs.docid[i]]}' appears twice in run '{rs.rankers[r]}' for "
                f"query '{rs.qids[q]}': duplicate docnos within one list are not supported")
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
                 docid=rs.docid[o], score=rs.score[o], rank=rs.rank[o])
    _analyse(out, lid[o])
    if by == "rank":
        # the kernel's order check is on scores; rank order is what W-RRF needs
        out.canonical = True
    return out

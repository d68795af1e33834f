"""Shared test helpers (golden decoding, frame building)."""
from __future__ import annotations

import numpy as np
import pandas as pd


def unhex(s: str) -> float:
    return float.fromhex(s)


def frames_from_rows(runs: dict, rankers=None) -> dict:
    """DataFrames in `rankers` order (the golden JSON stores dicts key-sorted)."""
    out = {}
    for r in (rankers or list(runs.keys())):
        rows = runs[r]
        df = pd.DataFrame(rows, columns=["qid", "docno", "rank", "score"])
        df.insert(1, "iter", "Q0")
        df["runid"] = r
        df["qid"] = df["qid"].astype(str)
        out[r] = df
    return out


def decode_fused(enc: dict) -> dict:
    return {q: [(d, unhex(s)) for d, s in lst] for q, lst in enc.items()}


def csr_from_rows(runs: dict, rankers: list, by_rank: bool = False):
    """Rows -> (qids, list_off, docid, score, rank, docnos) in file row order."""
    qids = sorted({row[0] for rows in runs.values() for row in rows})
    qi = {q: i for i, q in enumerate(qids)}
    docnos, did = [], {}
    lists = {(q, r): [] for q in range(len(qids)) for r in range(len(rankers))}
    for r, name in enumerate(rankers):
        for qid, doc, rank, score in runs[name]:
            lists[(qi[qid], r)].append((doc, rank, score))
    off = [0]
    docid, score, rank = [], [], []
    for q in range(len(qids)):
        for r in range(len(rankers)):
            items = lists[(q, r)]
            if by_rank:
                items = sorted(items, key=lambda x: x[1])
            for doc, rk, s in items:
                if doc not in did:
                    did[doc] = len(docnos)
                    docnos.append(doc)
                docid.append(did[doc])
                score.append(s)
                rank.append(rk)
            off.append(len(docid))
    return (qids, np.array(off, np.int64), np.array(docid, np.uint32),
            np.array(score, np.float64), np.array(rank, np.int32), np.array(docnos, object))


def first_seen_lists(qids, docnos, ud, uc, perm, fused, list_off, R):
    """Rebuild {qid: [(docno, score)]} in first-seen order from kernel/oracle outputs."""
    out = {}
    for qi, q in enumerate(qids):
        b = int(list_off[qi * R])
        n = int(uc[qi])
        p = perm[b:b + n].astype(np.int64)
        s = np.empty(n)
        s[p] = fused[b:b + n]
        out[q] = list(zip(docnos[ud[b:b + n]].tolist(), s.tolist()))
    return out


def sorted_lists(qids, docnos, ud, uc, perm, fused, list_off, R):
    out = {}
    for qi, q in enumerate(qids):
        b = int(list_off[qi * R])
        n = int(uc[qi])
        p = perm[b:b + n].astype(np.int64)
        out[q] = list(zip(docnos[ud[b + p]].tolist(), fused[b:b + n].tolist()))
    return out

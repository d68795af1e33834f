"""Drop-in for the reference's research fusion scripts.

ProbFuse.py — probFuse: segment probabilities trained on judged runs
(train_probfuse, ProbFuse.py:92-133), then S_d = sum over runs of P_r[k-1] / k
with k the rank's segment (build_probfuse_run, ProbFuse.py:136-187).
QPPrrf_argmax.py — (weighted) RRF with weight * (1 / (k + rank)) per row
(build_rrf_run, QPPrrf_argmax.py:53-76) and argmax-QPP ranker selection
(build_adaptive_run, QPPrrf_argmax.py:33-51).

The fusions run on the device through the same join + sort kernels as the main
path (qf_fuse_probfuse with QF_PROBFUSE, qf_fuse with QF_WRRF_MUL): the per-row
contribution differs, the first-seen accumulation order (runs in dict order,
rows in file order) and the stable score-descending sort are the reference's.
train_probfuse is counting over the training runs and argmax selection is a
copy of one run's rows: both stay on the host (numpy / the reference's own
pandas calls).  Same function names, arguments, return values and file formats
as the reference scripts.
"""
from __future__ import annotations

import math
import os
from collections import defaultdict
from typing import Dict, List, Optional

import numpy as np
import pandas as pd

from . import engine
from .runset import pack_frames

__all__ = ["pos_to_segment", "load_runs", "train_probfuse", "build_probfuse_run",
           "write_runfile", "load_qpp_estimates", "load_argmax_runs", "build_rrf_run",
           "build_adaptive_run"]


# ------------------------------------------------------------- probFuse ------

def pos_to_segment(pos, L, x):
    """Map 1-indexed rank position to 1..x segment index (ProbFuse.py:30-39)."""
    if pos <= 0:
        pos = 1
    k = math.ceil((pos * x) / float(L))
    return int(min(max(k, 1), x))


def _segments(pos: np.ndarray, L: int, x: int) -> np.ndarray:
    """pos_to_segment over an int64 array, in integers (exact for |pos * x| < 2^53)."""
    p = np.maximum(pos.astype(np.int64), 1)
    return np.clip(-((-p * x) // L), 1, x)


def load_runs(res_path: str) -> Dict[str, pd.DataFrame]:
    """ProbFuse.py:42-58: every *.norm.res in sorted order, qid / docno as str."""
    from . import fastio
    files = sorted(f for f in os.listdir(res_path) if f.endswith(".norm.res"))
    if not files:
        raise ValueError(f"No .res files found in {res_path}")
    names = [f.replace(".norm.res", "") for f in files]
    _, frames = fastio.parse_runs([os.path.join(res_path, f) for f in files], names)
    return frames


def train_probfuse(runs_train, qrels_train_dict, x=25, L=100, variant="judged", eps=0.0):
    """P_probs[ranker] = x segment probabilities (ProbFuse.py:92-133), counted with numpy."""
    P_probs = {}
    for ranker, df in runs_train.items():
        qid = df["qid"].astype(str).to_numpy()
        doc = df["docno"].astype(str).to_numpy()
        k = _segments(df["rank"].to_numpy(dtype=np.int64), L, x) - 1
        lab = np.array([qrels_train_dict[q][d] if q in qrels_train_dict and
                        d in qrels_train_dict[q] else -(1 << 62) for q, d in zip(qid, doc)],
                       dtype=np.int64)
        judged = lab != -(1 << 62)
        total = np.bincount(k, minlength=x)
        rel = np.bincount(k[judged & (lab > 0)], minlength=x)
        nonrel = np.bincount(k[judged & (lab <= 0)], minlength=x)
        probs = [0.0] * x
        for s in range(x):
            if variant.lower() == "all":
                denom, num = int(total[s]), int(rel[s])
            elif variant.lower() == "judged":
                denom, num = int(rel[s] + nonrel[s]), int(rel[s])
            else:
                raise ValueError("variant must be 'all' or 'judged'")
            probs[s] = float(num) / float(denom) if denom > 0 else eps
        P_probs[ranker] = probs
    return P_probs


def _qid_key(q: str):
    return int(q) if q.isdigit() else q


def _frame(qids, docs, scores, tag) -> pd.DataFrame:
    n = np.array([len(d) for d in docs], dtype=np.int64)
    rank = np.concatenate([np.arange(1, m + 1, dtype=np.int64) for m in n]) if len(n) else \
        np.zeros(0, np.int64)
    return pd.DataFrame({
        "qid": np.repeat(np.asarray(qids, dtype=object), n),
        "iter": "Q0",
        "docno": np.concatenate(docs) if docs else np.zeros(0, object),
        "rank": rank,
        "score": np.concatenate(scores) if scores else np.zeros(0, np.float64),
        "runid": tag}, columns=["qid", "iter", "docno", "rank", "score", "runid"])


def _device_fuse(rs, method: str, weights=None, k: int = 60, seg=None):
    import torch
    dev = engine.require_device()
    d = rs.to_device()
    wd = None if weights is None else torch.from_numpy(np.ascontiguousarray(weights)).to(dev)
    kw = {}
    if seg is not None:
        table, x, L = seg
        kw = dict(seg_prob=torch.from_numpy(np.ascontiguousarray(table, np.float64)).to(dev),
                  n_segments=x, seg_len=L)
    out = engine.fuse(d["list_off"], d["docid"], d["score"], rs.n_rankers, [method], rrf_k=k,
                      weights=wd, rank=d["rank"], max_entries=rs.max_entries(), **kw)
    counts = out.union_count.cpu().numpy()[:rs.n_queries]
    bad = np.nonzero(counts < 0)[0]
    if bad.size:
        from ._lib import QF_QSTATUS
        code = int(counts[bad[0]])
        raise ValueError(f"query '{rs.qids[bad[0]]}': {QF_QSTATUS.get(code, code)}")
    E = rs.n_entries
    return (counts, out.union_docid.cpu().numpy()[:E].view(np.uint32),
            out.perm.cpu().numpy()[0, :E].view(np.uint16), out.fused.cpu().numpy()[0, :E])


def _ranked(rs, counts, udoc, perm, fused, qi):
    b, n = int(rs.list_off[qi * rs.n_rankers]), int(counts[qi])
    p = perm[b:b + n].astype(np.int64)
    return rs.docnos[udoc[b + p]], fused[b:b + n]


def build_probfuse_run(runs_test, P_probs, x=25, L=100, run_tag="probFuse") -> pd.DataFrame:
    """Fused run DataFrame: S_d = sum_m P_m[k-1] / k (ProbFuse.py:136-187), on device."""
    rankers = list(runs_test.keys())
    all_qids = set()
    for r in rankers:
        all_qids.update(runs_test[r]["qid"].astype(str).unique())
    all_qids = sorted(all_qids, key=_qid_key)
    if not all_qids:
        return _frame([], [], [], run_tag)
    rs = pack_frames(runs_test)
    table = np.zeros((len(rankers), x), np.float64)
    for i, r in enumerate(rankers):
        if r in P_probs:
            table[i] = np.asarray(P_probs[r], np.float64)[:x]
    counts, udoc, perm, fused = _device_fuse(rs, "probfuse", seg=(table, x, L))
    index = {q: i for i, q in enumerate(rs.qids)}
    docs, scores = [], []
    for q in all_qids:
        d, s = _ranked(rs, counts, udoc, perm, fused, index[q])
        docs.append(d)
        scores.append(s)
    return _frame(all_qids, docs, scores, run_tag)


def write_runfile(df, path):
    """ProbFuse.py:190-195: rows sorted by (qid, rank), "%.6f" scores."""
    df_sorted = df.sort_values(["qid", "rank"])
    with open(path, "w") as fout:
        fout.write("".join(f"{q} Q0 {d} {int(r)} {float(s):.6f} {t}\n" for q, d, r, s, t in zip(
            df_sorted["qid"], df_sorted["docno"], df_sorted["rank"], df_sorted["score"],
            df_sorted["runid"])))
    print(f"Saved fused run to: {path}")


# ------------------------------------------------------- QPPrrf_argmax -------

def load_qpp_estimates(qpp_path):
    """{qid: {ranker: [qpp...]}} from *.mmnorm.qpp (QPPrrf_argmax.py:9-29)."""
    qpp_data = defaultdict(dict)
    files = [os.path.join(qpp_path, f) for f in os.listdir(qpp_path) if f.endswith(".mmnorm.qpp")]
    for f in files:
        ranker = os.path.basename(f).replace(".res.mmnorm.qpp", "")
        with open(f, "r") as fin:
            for line in fin:
                parts = line.strip().split("\t")
                if len(parts) < 2:
                    continue
                qpp_data[parts[0]][ranker] = [float(v) for v in parts[1:]]
    return qpp_data


def load_argmax_runs(res_path):
    """QPPrrf_argmax.py:31-41 load_runs: *.100.res, pandas' own dtypes."""
    runs = {}
    for f in [f for f in os.listdir(res_path) if f.endswith(".100.res")]:
        runs[f.replace(".res", "")] = pd.read_csv(
            os.path.join(res_path, f), sep=r"\s+",
            names=["qid", "iter", "docno", "rank", "score", "runid"])
    return runs


def build_rrf_run(runs, k=60, qpp_data=None, qpp_method_index=None) -> pd.DataFrame:
    """(Weighted) RRF as QPPrrf_argmax.py:53-76 forms it: for each qid of the first
    run, sum over runs and rows (file order) of weight * (1 / (k + rank)), weight =
    qpp[str(qid)][ranker][index] (0.0 when missing), 1.0 unweighted; on device."""
    rankers = list(runs.keys())
    tag = "Weighted-RRF" if qpp_data else "RRF"
    first = runs[rankers[0]]["qid"]
    if not pd.api.types.is_integer_dtype(first.dtype):
        # the reference selects rows with df["qid"] == int(qid): int() raises on a
        # non-numeric qid, and no row of a string column equals an int
        for q in first.unique():
            int(q)
        return _frame([], [], [], tag)
    order = list(first.unique())
    rs = pack_frames(runs)
    index = {q: i for i, q in enumerate(rs.qids)}
    w = np.ones(rs.n_queries * rs.n_rankers, np.float64)
    if qpp_data and qpp_method_index is not None:
        for qi, q in enumerate(rs.qids):
            for ri, r in enumerate(rankers):
                try:
                    w[qi * rs.n_rankers + ri] = qpp_data[str(q)][r][qpp_method_index]
                except KeyError:
                    w[qi * rs.n_rankers + ri] = 0.0
    counts, udoc, perm, fused = _device_fuse(rs, "wrrf_mul", weights=w, k=k)
    int_docs = all(pd.api.types.is_integer_dtype(runs[r]["docno"].dtype) for r in rankers)
    qids, docs, scores = [], [], []
    for q in order:
        qi = index.get(str(q))
        if qi is None or counts[qi] == 0:
            continue
        d, s = _ranked(rs, counts, udoc, perm, fused, qi)
        qids.append(q)
        docs.append(np.array([int(x) for x in d], dtype=object) if int_docs else d)
        scores.append(s)
    return _frame(qids, docs, scores, tag)


def build_adaptive_run(qpp_data, runs, qpp_method_index=0) -> pd.DataFrame:
    """Argmax-QPP selection (QPPrrf_argmax.py:33-51): per query the run whose QPP
    column is largest (first in dict order on ties), re-ranked by score.  A row
    copy, so it stays on the host with the reference's own pandas calls."""
    records = []
    for qid, ranker_scores in qpp_data.items():
        if not ranker_scores:
            continue
        selected = max(ranker_scores.items(), key=lambda x: x[1][qpp_method_index])[0]
        df = runs[selected.split(".res")[0]]
        records.append(df[df["qid"] == int(qid)])
    if records:
        out = pd.concat(records)
        out = out.sort_values(["qid", "score"], ascending=[True, False])
        out["rank"] = out.groupby("qid").cumcount() + 1
        return out
    return pd.DataFrame(columns=["qid", "iter", "docno", "rank", "score", "runid"])

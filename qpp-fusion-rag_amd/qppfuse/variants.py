"""Drop-in for the reference's research fusion scripts.

ProbFuse.py — probFuse: segment probabilities trained on judged runs
(train_probfuse, ProbFuse.py:92-133), then S_d = sum over runs of P_r[k-1] / k
with k the rank's segment (build_probfuse_run, ProbFuse.py:136-187).
QPPrrf_argmax.py — (weighted) RRF with weight * (1 / (k + rank)) per row
(build_rrf_run, QPPrrf_argmax.py:53-76) and argmax-QPP ranker selection
(build_adaptive_run, QPPrrf_argmax.py:33-51).
10_oracle_baseline.py — the oracle upper bound: per query the ranker with the
best per-query metric (compute_oracle_run, :152-201), its evaluation and the
selection statistics (:204-254).
The scripts' evaluation mains — parse_measures (ProbFuse.py:198-222, AP(rel=2)
for "map"), the argmax / weighted-RRF run lists (QPPrrf_argmax.py:137-160) and
pyterrier's Experiment table over them — as parse_measures, argmax_runs and
experiment (means on the device through IREvaluator; pyterrier is absent here,
so its aggregation is restated as trec_eval's default — the run's queries that
have qrels — and that parity is unpinned).

The fusions and the per-query metrics run on the device through the same join + sort kernels as the main
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
from typing import Dict, List, NamedTuple, Optional

import numpy as np
import pandas as pd

from . import engine
from .runset import pack_frames

__all__ = ["pos_to_segment", "load_runs", "train_probfuse", "build_probfuse_run",
           "write_runfile", "load_qpp_estimates", "load_argmax_runs", "build_rrf_run",
           "build_adaptive_run", "load_all_runs", "parse_metric", "compute_per_query_scores",
           "compute_oracle_run", "evaluate_run", "analyze_oracle_selections", "model_name_dict",
           "Measure", "parse_measures", "parse_argmax_measures", "experiment", "argmax_runs"]


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
            out.perm.cpu().numpy()[0, :E].view(np.uint32 if out.wide else np.uint16),
            out.fused.cpu().numpy()[0, :E])


def _ranked(rs, counts, udoc, perm, fused, qi):
    b, n = int(rs.list_off[qi * rs.n_rankers]), int(counts[qi])
    p = perm[b:b + n].astype(np.int64)
    return rs.docnos[udoc[b + p]], fused[b + p]  # scores by u, ranked through perm


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


# ------------------------------------------------- 10_oracle_baseline --------

def load_all_runs(runs_dir, use_normalized: bool = False):
    """{ranker: {qid: [(docid, score)]}} with every list sorted by score descending
    (stable), as 10_oracle_baseline.py:56-88 loads *.res or *.norm.res."""
    from pathlib import Path
    from .data_utils import load_run_file
    runs_dir = Path(runs_dir)
    suffix = ".norm.res" if use_normalized else ".res"
    files = sorted(f for f in runs_dir.glob(f"*{suffix}")
                   if use_normalized or ".norm." not in f.name)
    runs = {}
    for f in files:
        name = f.name.replace(".norm.res", "") if use_normalized else f.stem
        runs[name] = {qid: [(d, s) for d, s, _ in sorted(docs, key=lambda t: -t[1])]
                      for qid, docs in load_run_file(f).items()}
    return runs


def parse_metric(metric_str: str) -> str:
    """Selection metric name (10_oracle_baseline.py:91-115): ndcg[@k] (k=10),
    map/ap, [m]rr[@k] (k=10), recall[@k] / r@k (k=10); the ir_measures object's
    string form ("nDCG@10", "AP", "RR@10", "R@10") is what qppfuse.evaluation takes."""
    m = metric_str.lower().strip()
    cut = (lambda: int(m.split("@")[1])) if "@" in m else (lambda: 10)
    if "ndcg" in m:
        return f"nDCG@{cut()}"
    if m in ("map", "ap"):
        return "AP"
    if "rr" in m or "mrr" in m:
        return f"RR@{cut()}"
    if "recall" in m or m.startswith("r@"):
        return f"R@{cut()}"
    raise ValueError(f"Unknown metric: {metric_str}")


def _pack_lists(lists):
    """[{docno: score}] -> docnos (sorted), off, docid, score; each list score-descending."""
    all_docs = np.asarray(sorted({d for dd in lists for d in dd}), dtype=object)
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    ids, scs = [], []
    for i, dd in enumerate(lists):
        names = np.asarray(list(dd.keys()), dtype=object)
        sc = np.fromiter(dd.values(), dtype=np.float64, count=len(dd))
        o = np.argsort(-sc, kind="stable")
        ids.append(np.searchsorted(all_docs, names).astype(np.uint32)[o])
        scs.append(sc[o])
        off[i + 1] = off[i] + len(dd)
    cat = lambda parts, dt: np.concatenate(parts) if parts else np.zeros(0, dt)
    return all_docs, off, cat(ids, np.uint32), cat(scs, np.float64)


def compute_per_query_scores(runs, qrels, metric):
    """{ranker: {qid: value}} (10_oracle_baseline.py:118-149): every (ranker, qid)
    list of every ranker goes to ONE qf_eval launch; a query without qrels (or
    without documents) gets no value, as ir_measures.iter_calc yields none."""
    import torch
    from .evaluation import evaluate_device, pack_qrels
    name = metric if isinstance(metric, str) else str(metric)
    keys, lists = [], []
    for ranker, run in runs.items():
        for qid, docs in run.items():
            keys.append((ranker, str(qid)))
            lists.append({str(d): float(s) for d, s in docs})  # the last repeat wins
    out = {r: {} for r in runs}
    if not lists:
        return out
    dev = engine.require_device()
    docnos, off, docid, score = _pack_lists(lists)
    qs = pack_qrels({str(q): r for q, r in qrels.items()}, [q for _, q in keys], docnos)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    v = evaluate_device(t(off), 1, None, t(docid.view(np.int32)), None, t(score), 0, 1,
                        len(lists), qs.to_device(dev), qs.max_per_query, [name],
                        text_scores=False)[0, :, 0].cpu().numpy()
    for (ranker, qid), x in zip(keys, v):
        if not np.isnan(x):
            out[ranker][qid] = float(x)
    return out


def _select_best(runs, qrels, per_query_scores):
    """The selection loop of compute_oracle_run (10_oracle_baseline.py:171-199):
    sorted qids judged in qrels, rankers in dict order, strictly greater wins,
    best_score starts at -1."""
    all_qids = set(qrels.keys())
    for run in runs.values():
        all_qids.update(run.keys())
    all_qids &= set(qrels.keys())
    oracle_run, selections = {}, {}
    for qid in sorted(all_qids):
        best, best_ranker = -1, None
        for ranker in runs:
            if qid in per_query_scores[ranker]:
                sc = per_query_scores[ranker][qid]
                if sc > best:
                    best, best_ranker = sc, ranker
        if best_ranker and qid in runs[best_ranker]:
            oracle_run[qid] = runs[best_ranker][qid]
            selections[qid] = best_ranker
    return oracle_run, selections


def compute_oracle_run(runs, qrels, metric):
    """(oracle_run {qid: [(docid, score)]}, selections {qid: ranker})."""
    return _select_best(runs, qrels, compute_per_query_scores(runs, qrels, metric))


def evaluate_run(run, qrels, metrics) -> Dict[str, float]:
    """{metric: mean over the evaluated queries} (10_oracle_baseline.py:204-214) on device."""
    from .evaluation import IREvaluator
    names = [m if isinstance(m, str) else str(m) for m in metrics]
    return {k: float(v) for k, v in IREvaluator(names).evaluate(run, qrels).items()}


def analyze_oracle_selections(selections, per_query_scores):
    """Selection counts / percentages and the mean relative gain of the selected
    ranker over the mean of the others (10_oracle_baseline.py:217-254)."""
    counts = defaultdict(int)
    for ranker in selections.values():
        counts[ranker] += 1
    total = len(selections)
    gains = []
    for qid, best_ranker in selections.items():
        best = per_query_scores[best_ranker].get(qid, 0)
        others = [per_query_scores[r].get(qid, 0) for r in per_query_scores if r != best_ranker]
        if others:
            avg = np.mean(others)
            if avg > 0:
                gains.append((best - avg) / avg * 100)
    return {"selection_counts": dict(counts),
            "selection_percentages": {r: c / total * 100 for r, c in counts.items()},
            "n_queries": total,
            "avg_improvement_over_others": np.mean(gains) if gains else 0,
            "max_improvement": max(gains) if gains else 0}


# ------------------------------------------------ the scripts' evaluation mains ------

# QPPrrf_argmax.py:9 — the names its per-column runs carry
model_name_dict = {0: "SMV", 1: "Sigma_max", 2: "Sigma(%)", 3: "NQC", 4: "UEF", 5: "RSD",
                   6: "QPP-PRP", 7: "WIG", 8: "SCNQC", 9: "QV-NQC", 10: "DM", 11: "NQA-QPP",
                   12: "BERTQPP"}


class Measure(NamedTuple):
    """One pyterrier measure: its printed name, the IREvaluator metric and the
    relevance level (judged grades below it count as non-relevant)."""
    name: str
    metric: str
    rel: int = 1


def parse_measures(metrics_list) -> List[Measure]:
    """ProbFuse.py:198-222: map -> AP(rel=2), ndcg[@k] -> nDCG[@k], recip_rank / rr
    -> RR, p<k> -> P@k; anything else raises ValueError."""
    out = []
    for m in metrics_list:
        mlow = m.lower()
        if mlow == "map":
            out.append(Measure("AP(rel=2)", "AP", 2))
        elif mlow.startswith("ndcg"):
            if "@" in mlow:
                k = int(mlow.split("@")[1])
                out.append(Measure(f"nDCG@{k}", f"nDCG@{k}"))
            else:
                out.append(Measure("nDCG", "nDCG"))
        elif mlow in ("recip_rank", "rr"):
            out.append(Measure("RR", "RR"))
        elif mlow.startswith("p"):
            try:
                k = int(mlow[1:])
            except ValueError:
                raise ValueError(f"Unsupported metric {m}") from None
            out.append(Measure(f"P@{k}", f"P@{k}"))
        else:
            raise ValueError(f"Unsupported metric {m}")
    return out


def parse_argmax_measures(metrics) -> List[Measure]:
    """QPPrrf_argmax.py:119-131: map -> AP(rel=2), a name containing "ndcg@10" ->
    nDCG@k, recip_rank -> RR; other names are skipped, as there."""
    out = []
    for m in metrics:
        if m.lower() == "map":
            out.append(Measure("AP(rel=2)", "AP", 2))
        elif "ndcg@10" in m.lower():
            k = int(m.split("@")[1]) if "@" in m else None
            out.append(Measure(f"nDCG@{k}", f"nDCG@{k}") if k else Measure("nDCG", "nDCG"))
        elif m.lower() == "recip_rank":
            out.append(Measure("RR", "RR"))
    return out


def experiment(runs, qrels, measures, names) -> pd.DataFrame:
    """pyterrier's Experiment(runs, qrels, topics, eval_metrics, names) table as the
    scripts print it: one row per run (`name`, then one mean per measure).  Runs
    are DataFrames (qid, docno, score) or {qid: [(docno, score)]}; qrels a
    {qid: {docno: grade}} dict or a (qid, docno, label) DataFrame."""
    from .evaluation import IREvaluator
    if isinstance(qrels, pd.DataFrame):
        qrels = IREvaluator._convert_qrels(qrels)
    measures = [m if isinstance(m, Measure) else Measure(str(m), str(m)) for m in measures]
    by_rel: Dict[int, List[Measure]] = defaultdict(list)
    for m in measures:
        by_rel[int(m.rel)].append(m)
    leveled = {t: (qrels if t <= 1 else
                   {q: {d: (g if g >= t else 0) for d, g in docs.items()}
                    for q, docs in qrels.items()})
               for t in by_rel}
    rows = []
    for run, name in zip(runs, names):
        row = {"name": name}
        for t, ms in by_rel.items():
            vals = IREvaluator([m.metric for m in ms]).evaluate(run, leveled[t])
            for m in ms:
                row[m.name] = float(vals[m.metric])
        rows.append(row)
    return pd.DataFrame(rows, columns=["name"] + [m.name for m in measures])


def argmax_runs(strategy: str, runs, qpp_data):
    """The runs and names QPPrrf_argmax.py's main() evaluates (:137-160): per QPP
    column an adaptive (argmax) or weighted-RRF run, or one plain RRF run, then
    every input run as a baseline."""
    sample_scores = next(iter(next(iter(qpp_data.values())).values()))
    n = len(sample_scores)
    all_runs, all_names = [], []
    if strategy == "adaptive":
        for i in range(n):
            all_runs.append(build_adaptive_run(qpp_data, runs, qpp_method_index=i))
            all_names.append(f"Adaptive-QPP-{model_name_dict[i]}")
    elif strategy == "wrrf":
        for i in range(n):
            all_runs.append(build_rrf_run(runs, qpp_data=qpp_data, qpp_method_index=i))
            all_names.append(f"Weighted-RRF-QPP-{model_name_dict[i]}")
    elif strategy == "rrf":
        all_runs.append(build_rrf_run(runs))
        all_names.append("RRF")
    else:
        raise ValueError(f"strategy must be adaptive, rrf or wrrf, not {strategy!r}")
    all_runs.extend(runs.values())
    all_names.extend(runs.keys())
    return all_runs, all_names

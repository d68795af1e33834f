"""IR evaluation of (fused) runs on MI355X — the metrics step of the reference.

Mirrors src/evaluation/ir_evaluator.py (IREvaluator :40-150) and the way
scripts/06_eval_fusion.py:42-140 uses it on the fused .res files: the metrics
config.evaluation.ir_metrics names (config/defaults.yaml:224-234), computed
with trec_eval semantics (ir_measures' default backend): documents ranked by
score descending, ties by docno descending; relevant = rel >= 1; nDCG gains =
rel levels.  The work runs in the HIP kernel qf_eval (csrc/qf_eval.hip); this
module packs runs and qrels into its CSR layout.  There is no CPU path.
"""
from __future__ import annotations

import re
from collections.abc import Mapping
from operator import itemgetter
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import pandas as pd

from . import _lib, engine
from .config import config
from .data_utils import load_qrels, load_run_file

__all__ = ["IREvaluator", "parse_measure", "load_qrels", "load_run_file", "QrelSet",
           "pack_qrels", "evaluate_device"]

_KINDS = {"ndcg": _lib.EVAL_NDCG, "rr": _lib.EVAL_RR, "r": _lib.EVAL_R, "p": _lib.EVAL_P,
          "ap": _lib.EVAL_AP}
_NO_CUT = 1 << 30


def parse_measure(name: str) -> Tuple[int, int]:
    """'nDCG@10' -> (QF_EVAL_NDCG, 10); 'AP' / 'RR' without a cutoff -> whole list."""
    m = re.fullmatch(r"\s*([A-Za-z]+)\s*(?:@\s*(\d+))?\s*", name)
    if not m or m.group(1).lower() not in _KINDS:
        raise ValueError(f"unsupported measure '{name}' (nDCG@k, RR@k, R@k, P@k, AP)")
    kind = _KINDS[m.group(1).lower()]
    if m.group(2) is None:
        if kind in (_lib.EVAL_R, _lib.EVAL_P):
            raise ValueError(f"measure '{name}' needs a cutoff")
        return kind, _NO_CUT if kind != _lib.EVAL_AP else 0
    k = int(m.group(2))
    if k < 1:
        raise ValueError(f"measure '{name}': cutoff must be >= 1")
    return kind, k


class QrelSet:
    """Qrels in the run's query order: CSR of (docid ascending, rel) per query."""

    def __init__(self, off: np.ndarray, docid: np.ndarray, rel: np.ndarray):
        self.off, self.docid, self.rel = off, docid, rel
        self.max_per_query = int(np.max(np.diff(off))) if len(off) > 1 else 0

    def to_device(self, device):
        import torch
        return (torch.from_numpy(self.off).to(device),
                torch.from_numpy(self.docid.view(np.int32)).to(device),
                torch.from_numpy(self.rel).to(device))


def pack_qrels(qrels: Dict[str, Dict[str, int]], qids: Sequence[str],
               docnos: np.ndarray) -> QrelSet:
    """Map qrels onto the run's queries and docno ids (docnos sorted ascending).

    Judged documents absent from the run keep their place in the counts (they
    are relevant but never retrieved) under the reserved id 0xFFFFFFFF."""
    offs = [0]
    ids: List[np.ndarray] = []
    rels: List[np.ndarray] = []
    for qid in qids:
        judged = qrels.get(qid, {})
        if not judged:
            offs.append(offs[-1])
            continue
        names = np.asarray(list(judged.keys()), dtype=object)
        rv = np.fromiter(judged.values(), dtype=np.int32, count=len(judged))
        pos = np.searchsorted(docnos, names)
        pos_c = np.minimum(pos, max(len(docnos) - 1, 0))
        found = (pos < len(docnos)) & (docnos[pos_c] == names) if len(docnos) else \
            np.zeros(len(names), bool)
        d = np.where(found, pos_c, 0xFFFFFFFF).astype(np.uint32)
        o = np.argsort(d, kind="stable")
        ids.append(d[o])
        rels.append(rv[o])
        offs.append(offs[-1] + len(judged))
    off = np.asarray(offs, dtype=np.int64)
    docid = np.concatenate(ids) if ids else np.zeros(0, np.uint32)
    rel = np.concatenate(rels) if rels else np.zeros(0, np.int32)
    return QrelSet(off, docid, rel)


def _ranked_index(qbase, counts, perm):
    """(source, destination) indices that put every query's list in rank order at
    its own slots: destination qbase[q] + i takes source qbase[q] + perm[qbase[q] + i]."""
    counts = np.maximum(np.asarray(counts, np.int64), 0)
    qb = np.asarray(qbase, np.int64)
    dst = np.repeat(qb, counts) + (np.arange(int(counts.sum()), dtype=np.int64)
                                   - np.repeat(np.cumsum(counts) - counts, counts))
    return np.repeat(qb, counts) + perm[dst].astype(np.int64), dst


def evaluate_device(q_base, base_stride: int, q_count, docid, perm, score, out_stride: int,
                    n_runs: int, n_queries: int, qrels_dev, max_qrels: int,
                    measures: Sequence[str], text_scores: bool = True):
    """qf_eval on device buffers -> float64 tensor [n_runs, n_queries, n_measures]."""
    import torch
    dev = engine.require_device()
    spec = [parse_measure(m) for m in measures]
    if len(spec) > _lib.EVAL_MAX_METRICS:
        raise ValueError(f"at most {_lib.EVAL_MAX_METRICS} measures per call")
    if max_qrels > _lib.EVAL_MAX_QRELS:
        raise ValueError(f"{max_qrels} judged documents in one query exceed "
                         f"{_lib.EVAL_MAX_QRELS}")
    kind = np.asarray([k for k, _ in spec], dtype=np.int32)
    cut = np.asarray([c for _, c in spec], dtype=np.int32)
    out = torch.empty((n_runs, n_queries, len(spec)), dtype=torch.float64, device=dev)
    qo, qd, qr = qrels_dev
    p = engine._ptr
    _lib.call("qf_eval", int(n_queries), p(q_base), int(base_stride), p(q_count), p(docid),
              p(perm), p(score), int(out_stride), int(n_runs), int(bool(text_scores)), p(qo),
              p(qd), p(qr), int(max_qrels), len(spec), kind.ctypes.data, cut.ctypes.data,
              p(out), engine._stream())
    return out


def _run_arrays(run) -> Tuple[List[str], np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """{qid: [(docno, score)]} / DataFrame -> qids, docnos (sorted), off, docid, score.

    Each query's list is ordered by score descending (stable), as
    scripts/06_eval_fusion.py:46-49 orders it before evaluation."""
    if isinstance(run, pd.DataFrame):
        q = run["qid" if "qid" in run else "query_id"].astype(str).to_numpy()
        d = run["docno" if "docno" in run else "doc_id"].astype(str).to_numpy()
        s = run["score"].to_numpy(dtype=np.float64)
        # later rows of a repeated (qid, docno) win, as the dict conversion does
        df = pd.DataFrame({"q": q, "d": d, "s": s}).drop_duplicates(["q", "d"], keep="last")
        groups = {k: list(zip(g["d"], g["s"])) for k, g in df.groupby("q", sort=False)}
        run = groups
    qids = [str(k) for k in run.keys()]
    fast = _run_arrays_flat(run, qids)
    if fast is not None:
        return fast
    per_q = []
    for qid in run:
        items = run[qid]
        if isinstance(items, Mapping):
            items = list(items.items())
        dd = {}
        for doc, sc in items:  # ir_measures' dict: a repeated docno keeps its last score
            dd[str(doc)] = float(sc)
        per_q.append(dd)
    all_docs = np.asarray(sorted({d for dd in per_q for d in dd}), dtype=object)
    off = np.zeros(len(per_q) + 1, dtype=np.int64)
    docid_parts, score_parts = [], []
    for i, dd in enumerate(per_q):
        names = np.asarray(list(dd.keys()), dtype=object)
        sc = np.fromiter(dd.values(), dtype=np.float64, count=len(dd))
        ids = np.searchsorted(all_docs, names).astype(np.uint32)
        o = np.argsort(-sc, kind="stable")
        docid_parts.append(ids[o])
        score_parts.append(sc[o])
        off[i + 1] = off[i] + len(dd)
    docid = np.concatenate(docid_parts) if docid_parts else np.zeros(0, np.uint32)
    score = np.concatenate(score_parts) if score_parts else np.zeros(0)
    return qids, all_docs, off, docid, score


def _coded_by_table(flat, n):
    """Rows whose docnos are the very str objects of the last table read_run_rows
    returned (load_run_file's rows, through the 06 script's per-query sort): their
    codes into the run's sorted docnos by object identity and the table's Arrow sort
    — (codes, sorted docnos), or None when any row holds another object."""
    from .fastio import docno_tables
    if not docno_tables or n == 0:
        return None
    tab = docno_tables[-1]
    if len(tab.objs) == 0:
        return None
    at = tab.id_index().get_indexer(np.fromiter(map(id, map(itemgetter(0), flat)), np.uint64, n))
    if at.min() < 0:                           # a row holds another object
        return None
    # (at: rows -> table positions; the table holds the objects, so no id is reused)
    srt = tab.sorted_order()                   # table positions, ascending strings
    used = np.zeros(len(srt), bool)
    used[at] = True
    srt = srt[used[srt]]                       # the run's docnos, ascending
    rank = np.empty(len(used), np.int64)
    rank[srt] = np.arange(len(srt))
    return rank[at], tab.objs[srt]


def _run_arrays_flat(run, qids):
    """_run_arrays for a run without a repeated (query, docno): the same arrays from
    one flat pass — docnos coded by identity with load_run_file's table when the rows
    hold its strings, else sorted and coded by pandas.factorize; each query's list
    ordered by a stable lexsort on (query, -score) unless already in that order —
    instead of per-query dicts and a binary search of every docno in the sorted
    table (C2's 14 M rows: ~1 min -> s).  None when a query repeats a docno (the
    dict semantics decide: the slow path)."""
    lists = []
    for qid in run:
        items = run[qid]
        lists.append(list(items.items()) if isinstance(items, Mapping) else items)
    lens = np.fromiter((len(x) for x in lists), dtype=np.int64, count=len(lists))
    n = int(lens.sum())
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    if n == 0:
        return qids, np.zeros(0, dtype=object), off, np.zeros(0, np.uint32), np.zeros(0)
    flat = [it for x in lists for it in x]
    sc = np.fromiter(map(float, map(itemgetter(1), flat)), dtype=np.float64, count=n)
    coded = _coded_by_table(flat, n)
    if coded is not None:
        codes, all_docs = coded
    else:
        docs = np.empty(n, dtype=object)
        docs[:] = [str(d) for d in map(itemgetter(0), flat)]
        codes, uniq = pd.factorize(docs, sort=True)
        all_docs = np.asarray(uniq, dtype=object)
    del flat
    qi = np.repeat(np.arange(len(lists), dtype=np.int64), lens)
    if np.unique(qi * len(all_docs) + codes).size != n:
        return None
    # stable: equal scores keep their list order (already so after 06's per-query sort)
    if n > 1 and bool(np.all((sc[1:] <= sc[:-1]) | (qi[1:] != qi[:-1]))):
        return qids, all_docs, off, codes.astype(np.uint32), sc
    order = np.lexsort((-sc, qi))
    return qids, all_docs, off, codes[order].astype(np.uint32), sc[order]


class IREvaluator:
    """ir_measures-style evaluator (src/evaluation/ir_evaluator.py:40-150) on device."""

    def __init__(self, metrics: Optional[List[str]] = None, text_scores: bool = False):
        self.metric_names = list(metrics or config.evaluation.ir_metrics)
        for m in self.metric_names:
            parse_measure(m)
        # True: score ties as in the "%.6f" text of a run file (what 06_eval_fusion
        # evaluates); False: the doubles as given (an in-memory run).
        self.text_scores = text_scores

    def _per_query_values(self, run, qrels) -> Tuple[List[str], np.ndarray]:
        import torch
        from .fusion import FusedRun
        dev = engine.require_device()
        if isinstance(qrels, pd.DataFrame):
            qrels = self._convert_qrels(qrels)
        if isinstance(run, FusedRun):
            qids, docnos = run._qids, run._docnos
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
            q_base = t(run._qbase.astype(np.int64))
            q_count = t(run._counts.astype(np.int32))
            if run._perm.dtype == np.uint32:  # wide (qf_fuse_wide): qf_eval's perm is
                # uint16, so the lists go over in rank order instead (perm NULL)
                g = _ranked_index(run._qbase, run._counts, run._perm)
                udoc, fz = np.zeros_like(run._udoc), np.zeros_like(run._fused)
                udoc[g[1]], fz[g[1]] = run._udoc[g[0]], run._fused[g[0]]
                docid, perm, score = t(udoc.view(np.int32)), None, t(fz)
            else:
                docid = t(run._udoc.view(np.int32))
                perm = t(run._perm.view(np.int16))
                score = t(run._fused)
            qs = pack_qrels(qrels, qids, docnos)
            vals = []
            for a in range(0, len(self.metric_names), _lib.EVAL_MAX_METRICS):
                names = self.metric_names[a:a + _lib.EVAL_MAX_METRICS]
                vals.append(evaluate_device(q_base, 1, q_count, docid, perm, score, 0, 1,
                                            len(qids), qs.to_device(dev), qs.max_per_query,
                                            names, self.text_scores)[0])
            return qids, torch.cat(vals, 1).cpu().numpy()
        qids, docnos, off, docid_h, score_h = _run_arrays(run)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        qs = pack_qrels(qrels, qids, docnos)
        vals = []
        for a in range(0, len(self.metric_names), _lib.EVAL_MAX_METRICS):
            names = self.metric_names[a:a + _lib.EVAL_MAX_METRICS]
            vals.append(evaluate_device(t(off), 1, None, t(docid_h.view(np.int32)), None,
                                        t(score_h), 0, 1, len(qids), qs.to_device(dev),
                                        qs.max_per_query, names, self.text_scores)[0])
        return qids, torch.cat(vals, 1).cpu().numpy()

    def evaluate(self, run, qrels, per_query: bool = False):
        """{metric: mean over evaluated queries}, or {metric: {qid: value}}."""
        qids, v = self._per_query_values(run, qrels)
        if per_query:
            return {m: {q: float(v[i, t]) for i, q in enumerate(qids) if not np.isnan(v[i, t])}
                    for t, m in enumerate(self.metric_names)}
        out = {}
        for t, m in enumerate(self.metric_names):
            col = v[:, t]
            col = col[~np.isnan(col)]
            out[m] = float(col.mean()) if col.size else 0.0
        return out

    def evaluate_multiple(self, runs: Dict[str, object], qrels) -> pd.DataFrame:
        rows = []
        for name, run in runs.items():
            r = self.evaluate(run, qrels)
            r["run_name"] = name
            rows.append(r)
        df = pd.DataFrame(rows).set_index("run_name")
        return df.sort_values(by=self.metric_names[0], ascending=False)

    @staticmethod
    def _convert_qrels(qrels: pd.DataFrame) -> Dict[str, Dict[str, int]]:
        out: Dict[str, Dict[str, int]] = {}
        qc = "qid" if "qid" in qrels else "query_id"
        dc = "docno" if "docno" in qrels else "doc_id"
        lc = "label" if "label" in qrels else "relevance"
        for q, d, l in zip(qrels[qc].astype(str), qrels[dc].astype(str), qrels[lc]):
            out.setdefault(q, {})[d] = int(l)
        return out

"""File loaders of the path (boundary only): .qpp scores, TREC runs, qrels.

Same results and errors as the reference's src/data_utils.py loaders
(load_qrels :175-197, load_run_file :204-231, load_run_as_dict :234-255,
load_qpp_scores :262-293).  Host text parsing — no compute to accelerate.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np
from pathlib import Path
from typing import Dict, List, Tuple, Union

PathLike = Union[str, Path]


def load_qrels(qrels_path: PathLike) -> Dict[str, Dict[str, int]]:
    """BEIR qrels TSV (header line skipped) -> {qid: {docid: rel}}."""
    out: Dict[str, Dict[str, int]] = defaultdict(dict)
    with open(qrels_path, "r") as fh:
        next(fh, None)
        for line in fh:
            f = line.strip().split("\t")
            if len(f) >= 3:
                out[f[0]][f[1]] = int(f[2])
    return dict(out)


def load_run_file(run_path: PathLike) -> Dict[str, List[Tuple[str, float, int]]]:
    """TREC run -> {qid: [(docid, score, rank)]} sorted by rank (stable), queries in
    first-appearance order (src/data_utils.py:204-231).  The file is parsed by the
    native loader (qfio, as load_runs: the same float() / int() values); a file it
    rejects (a line without exactly 6 fields — the reference skips lines with fewer
    and ignores fields past the sixth) takes the reference's line loop."""
    try:
        from .fastio import read_run_rows
        qids, docnos, rq, rd, rr, rsc = read_run_rows(str(run_path))
    except ValueError:  # a format the loader rejects: the reference's loop decides
        return _load_run_file_lines(run_path)
    if len(rq) == 0:
        return {}
    # queries by first appearance; rows of a query by rank, stable (file order)
    _, first = np.unique(rq, return_index=True)
    qorder = np.argsort(first, kind="stable")      # codes in first-appearance order
    pos = np.empty(len(first), np.int64)
    pos[qorder] = np.arange(len(first))
    pq = pos[rq]
    if bool(np.all(pq[1:] >= pq[:-1])) and bool(np.all((rr[1:] >= rr[:-1]) | (pq[1:] != pq[:-1]))):
        q_sorted, d_col, s_col, r_col = pq, docnos[rd].tolist(), rsc.tolist(), rr.tolist()
    else:  # (a file already grouped by query in rank order — every run file this
        # package writes — needs no sort: the stable sort below is the identity there)
        order = np.lexsort((rr, pq))                # stable: ties keep file order
        q_sorted = pq[order]
        d_col = docnos[rd[order]].tolist()
        s_col = rsc[order].tolist()
        r_col = rr[order].tolist()
    bounds = np.flatnonzero(np.diff(q_sorted)) + 1
    # millions of tuples: without the cyclic collector's passes over them (they hold
    # no cycles), 13 -> ~1.5 s for C2's 14 M rows
    import gc
    enabled = gc.isenabled()
    gc.disable()
    try:
        rows = list(zip(d_col, s_col, r_col))
        starts = [0] + bounds.tolist()
        ends = bounds.tolist() + [len(rows)]
        codes = qorder.tolist()
        return {str(qids[codes[i]]): rows[a:b] for i, (a, b) in enumerate(zip(starts, ends))}
    finally:
        if enabled:
            gc.enable()


def _load_run_file_lines(run_path: PathLike) -> Dict[str, List[Tuple[str, float, int]]]:
    """src/data_utils.py:218-231, line by line."""
    out: Dict[str, list] = defaultdict(list)
    with open(run_path, "r") as fh:
        for line in fh:
            f = line.strip().split()
            if len(f) >= 6:
                out[f[0]].append((f[2], float(f[4]), int(f[3])))
    for qid in out:
        out[qid].sort(key=lambda x: x[2])
    return dict(out)


def load_run_as_dict(run_path: PathLike) -> Dict[str, Dict[str, float]]:
    out: Dict[str, Dict[str, float]] = defaultdict(dict)
    with open(run_path, "r") as fh:
        for line in fh:
            f = line.strip().split()
            if len(f) >= 5:
                out[f[0]][f[2]] = float(f[4])
    return dict(out)


def load_qpp_scores(qpp_path: PathLike) -> Dict[str, Dict[str, List[float]]]:
    """Directory of <Retriever>.res.mmnorm.qpp -> {qid: {retriever: [13 floats]}}."""
    qpp_path = Path(qpp_path)
    files = list(qpp_path.glob("*.mmnorm.qpp"))
    if not files:
        raise FileNotFoundError(f"No .mmnorm.qpp files in {qpp_path}")
    out: Dict[str, Dict[str, List[float]]] = defaultdict(dict)
    for fp in files:
        retriever = fp.stem.replace(".res.mmnorm", "")
        with open(fp, "r") as fh:
            for line in fh:
                f = line.strip().split("\t")
                if len(f) < 2:
                    continue
                out[f[0]][retriever] = [float(x) for x in f[1:]]
    return dict(out)

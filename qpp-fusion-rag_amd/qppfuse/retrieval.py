"""Per-query min-max normalisation of run lists (.res -> .norm.res) on MI355X.

Mirrors BaseRetriever.normalize_scores (src/retrievers/base.py:60-73) and the
normalising branch of scripts/02_retrieve.py write_run (:65-82); the arithmetic
is the HIP kernel qf_minmax_per_query, which also emits the exact "%.6f"
rounding as int32 micro-units.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from . import engine


@dataclass
class RetrieverResult:
    """The retrievers' output record (src/retrievers/base.py:14-29): what write_run reads."""
    qid: str
    results: List[Tuple[str, float, int]]  # (docno, score, rank)
    retriever_name: str
    latency_ms: float = 0.0
    metadata: Dict[str, Any] = field(default_factory=dict)

    def to_trec_lines(self, run_name: Optional[str] = None) -> List[str]:
        name = run_name or self.retriever_name
        return [f"{self.qid} Q0 {d} {r} {s:.6f} {name}" for d, s, r in self.results]


def _run(lists: List[np.ndarray]):
    import torch
    dev = engine.require_device()
    lens = np.fromiter((len(x) for x in lists), dtype=np.int64, count=len(lists))
    off = np.zeros(len(lists) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    flat = np.concatenate(lists) if lists else np.zeros(0)
    if flat.size == 0:
        return [np.zeros(0)] * len(lists), [np.zeros(0, np.int32)] * len(lists)
    norm, micro = engine.minmax_per_query(torch.from_numpy(flat.astype(np.float64)).to(dev),
                                          torch.from_numpy(off).to(dev))
    norm, micro = norm.cpu().numpy(), micro.cpu().numpy()
    return ([norm[off[i]:off[i + 1]] for i in range(len(lists))],
            [micro[off[i]:off[i + 1]] for i in range(len(lists))])


def normalize_scores(results: List[Tuple[str, float, int]]) -> List[Tuple[str, float, int]]:
    """(s - min) / (max - min), range -> 1.0 when max == min; [] for []."""
    if not results:
        return []
    norm, _ = _run([np.array([s for _, s, _ in results], dtype=np.float64)])
    return [(d, float(v), r) for (d, _, r), v in zip(results, norm[0].tolist())]


def _fmt_micro(m: int) -> str:
    sign = "-" if m < 0 else ""
    m = abs(int(m))
    return f"{sign}{m // 1000000}.{m % 1000000:06d}"


def write_run(results: Dict, output_path: str, retriever_name: str,
              normalize: bool = False) -> None:
    """scripts/02_retrieve.py:65-82: {qid: RetrieverResult} -> TREC run file.

    Same contract as the reference: each value's ``.results`` list of (docno,
    score, rank) is read (any object with that attribute — the reference's own
    RetrieverResult included), the output directory is created first
    (``os.makedirs(dirname, exist_ok=True)``, so a bare file name raises
    FileNotFoundError as there), qids in the ``testN`` numeric order, and with
    ``normalize`` every list min-max normalised (base.py:60-73) — all lists in one
    qf_minmax_per_query launch, written from its exact "%.6f" micro-units.
    """
    os.makedirs(os.path.dirname(output_path), exist_ok=True)
    qids = sorted(results.keys(), key=lambda x: int(x.replace("test", "")) if x.startswith("test") else x)
    docs_of = [results[q].results for q in qids]
    micro = None
    if normalize:
        _, micro = _run([np.array([s for _, s, _ in d], dtype=np.float64) for d in docs_of])
    with open(output_path, "w") as fh:
        for i, qid in enumerate(qids):
            for j, (docno, score, rank) in enumerate(docs_of[i]):
                txt = _fmt_micro(micro[i][j]) if normalize else f"{score:.6f}"
                fh.write(f"{qid} Q0 {docno} {rank} {txt} {retriever_name}\n")
    print(f"[02_retrieve] Wrote {output_path}")

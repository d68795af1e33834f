"""Per-query min-max normalisation of run lists (.res -> .norm.res) on MI355X.

Mirrors BaseRetriever.normalize_scores (src/retrievers/base.py:60-73) and the
normalising branch of scripts/02_retrieve.py write_run (:65-82); the arithmetic
is the HIP kernel qf_minmax_per_query, which also emits the exact "%.6f"
rounding as int32 micro-units.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from . import engine


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


def write_run(results: Dict[str, List[Tuple[str, float, int]]], output_path: str,
              retriever_name: str, normalize: bool = False) -> None:
    """TREC run writer of scripts/02_retrieve.py; all lists normalised in one launch."""
    qids = sorted(results.keys(), key=lambda x: int(x.replace("test", "")) if x.startswith("test") else x)
    micro = None
    if normalize:
        _, micro = _run([np.array([s for _, s, _ in results[q]], dtype=np.float64) for q in qids])
    with open(output_path, "w") as fh:
        for i, qid in enumerate(qids):
            docs = results[qid]
            for j, (docno, score, rank) in enumerate(docs):
                txt = _fmt_micro(micro[i][j]) if normalize else f"{score:.6f}"
                fh.write(f"{qid} Q0 {docno} {rank} {txt} {retriever_name}\n")

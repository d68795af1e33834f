"""FusionMLP inference restated on the CPU — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py may import this module, and
only as the checker.  Restates, with numpy float32 arithmetic and independently
of the device code:
  * FusionMLP._filter_features (src/models/mlp_model.py:104-122): model input
    j*n_used + k = X[:, j*n_qpp + qpp_indices[k]], applied only when fewer than
    n_qpp indices are used (:260-261);
  * predict (:254-274): torch.FloatTensor(X) (float64 -> float32, round to
    nearest even), Linear -> ReLU -> Dropout (identity: model.eval()) ... ->
    Linear, softmax(dim=1), then BaseFusionModel._normalize_weights
    (src/models/base.py:120-125) with the same numpy calls.
The float32 operation order is the one csrc/qf_learn.hip fixes (products and
sums each rounded, i ascending from +0.0, then + bias; softmax with
exp(double(z - max)) rounded to float32 and an ascending sum), so the device
matches this bit for bit.  torch's CPU GEMM/softmax (and the MPS device the
reference trained on) round in other orders: tests/golden/mlp/ holds the
reference's own FusionMLP.predict outputs, which this restatement matches
within float32 rounding (tests/test_boundary_golden.py).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np


def input_columns(n_retrievers: int, n_qpp: int, qpp_indices: List[int]) -> np.ndarray:
    if len(qpp_indices) >= n_qpp:
        return np.arange(n_retrievers * n_qpp)
    return np.asarray([j * n_qpp + i for j in range(n_retrievers) for i in qpp_indices])


def forward_logits(layers, x32: np.ndarray) -> np.ndarray:
    h = x32
    for li, (W, b) in enumerate(layers):
        W = np.asarray(W, np.float32)
        acc = np.zeros((h.shape[0], W.shape[0]), np.float32)
        for i in range(W.shape[1]):
            acc = acc + h[:, i:i + 1] * W[None, :, i]  # float32 product, then float32 sum
        acc = acc + np.asarray(b, np.float32)[None, :]
        if li + 1 < len(layers):
            acc = np.where(acc < 0, np.float32(0), acc)  # ReLU
        h = acc
    return h


def softmax32(z: np.ndarray) -> np.ndarray:
    m = z.max(axis=1, keepdims=True)
    e = np.exp((z - m).astype(np.float64)).astype(np.float32)
    s = np.zeros(z.shape[0], np.float32)
    for o in range(z.shape[1]):
        s = s + e[:, o]
    return e / s[:, None]


def normalize_weights(weights: np.ndarray) -> np.ndarray:
    """src/models/base.py:120-125 (the same numpy ops; float32 in, float32 out)."""
    weights = np.clip(weights, 0, None)
    sums = weights.sum(axis=1, keepdims=True)
    sums[sums == 0] = 1
    return weights / sums


def predict(layers, retrievers: List[str], n_qpp: int, qpp_indices: List[int],
            X: np.ndarray) -> np.ndarray:
    """FusionMLP.predict(X) -> float32 [n, n_retrievers] weights."""
    cols = input_columns(len(retrievers), n_qpp, qpp_indices)
    x32 = np.asarray(X, np.float64)[:, cols].astype(np.float32)
    return normalize_weights(softmax32(forward_logits(layers, x32)))


def weights_dict(runs, qpp_data, model, retrievers=None) -> Dict[str, Dict[str, np.float32]]:
    """src/fusion.py:415-434 for a FusionMLP: {qid: {retriever: np.float32 weight}}."""
    retrievers = list(retrievers or model.retrievers)
    n_qpp = model.n_qpp
    all_qids = sorted(set.union(*[set(df["qid"].unique()) for df in runs.values()]))
    X = np.zeros((len(all_qids), n_qpp * len(retrievers)))
    for i, qid in enumerate(all_qids):
        for j, retriever in enumerate(retrievers):
            if qid in qpp_data and retriever in qpp_data[qid]:
                X[i, j * n_qpp:(j + 1) * n_qpp] = qpp_data[qid][retriever][:n_qpp]
    pw = predict(model.layers, retrievers, n_qpp, model.qpp_indices, X)
    return {qid: {r: w for r, w in zip(retrievers, pw[i])} for i, qid in enumerate(all_qids)}

"""LightGBM inference + learned-fusion weights restated on the CPU — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py may import this module, and
only as the checker.  Restates, independently of the device code:
  * lightgbm Booster.predict on a regression model (LightGBM >= 4, not installed
    here — parity with the library is unpinned): first best_iteration trees; per
    tree, from node 0, Tree::NumericalDecision (missing type from decision_type
    bits 2-3: None -> fval <= threshold; Zero -> |fval| <= kZeroThreshold takes
    the default side (bit 1); NaN -> NaN takes it; a NaN with another missing
    type is read as 0.0); raw score = sum of leaf values in tree order from 0.0.
  * MultiOutputLGBM.predict / PerRetrieverLGBM.predict (src/models/
    lightgbm_models.py:114-123, 232-241): one column per booster, then
    BaseFusionModel._normalize_weights (src/models/base.py:120-125) — with the
    same numpy calls, so it is bit-identical by construction.
  * learned_fusion's feature matrix (src/fusion.py:415-427).
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np

K_ZERO = float(np.float32(1e-35))  # LightGBM kZeroThreshold is a float


def tree_output(tree, x) -> float:
    if tree.num_leaves <= 1:
        return float(tree.leaf_value[0])
    node = 0
    while node >= 0:
        fv = float(x[int(tree.split_feature[node])])
        dt = int(tree.decision_type[node])
        missing = (dt >> 2) & 3
        if math.isnan(fv) and missing != 2:
            fv = 0.0
        if (missing == 1 and -K_ZERO <= fv <= K_ZERO) or (missing == 2 and math.isnan(fv)):
            go_left = bool(dt & 2)
        else:
            go_left = fv <= float(tree.threshold[node])
        node = int(tree.left_child[node] if go_left else tree.right_child[node])
    return float(tree.leaf_value[~node])


def booster_predict(booster, X: np.ndarray) -> np.ndarray:
    out = np.zeros(X.shape[0])
    for i in range(X.shape[0]):
        s = 0.0
        for t in booster.used_trees:
            s += tree_output(t, X[i])
        out[i] = s
    return out


def normalize_weights(weights: np.ndarray) -> np.ndarray:
    """BaseFusionModel._normalize_weights, src/models/base.py:120-125 (same numpy ops)."""
    weights = np.clip(weights, 0, None)
    sums = weights.sum(axis=1, keepdims=True)
    sums[sums == 0] = 1
    return weights / sums


def model_predict(model, X: np.ndarray) -> np.ndarray:
    raw = np.column_stack([booster_predict(b, X) for b in model.boosters])
    return normalize_weights(raw)


def feature_matrix(qids: List[str], qpp_data, retrievers: List[str], n_qpp: int) -> np.ndarray:
    """src/fusion.py:421-427."""
    X = np.zeros((len(qids), n_qpp * len(retrievers)))
    for i, qid in enumerate(qids):
        for j, retriever in enumerate(retrievers):
            if qid in qpp_data and retriever in qpp_data[qid]:
                scores = qpp_data[qid][retriever]
                X[i, j * n_qpp:(j + 1) * n_qpp] = scores[:n_qpp]
    return X


def weights_dict(runs, qpp_data, model, retrievers=None) -> Dict[str, Dict[str, float]]:
    """src/fusion.py:415-434: {qid: {retriever: weight}}."""
    retrievers = retrievers or model.retrievers
    all_qids = sorted(set.union(*[set(df["qid"].unique()) for df in runs.values()]))
    X = feature_matrix(all_qids, qpp_data, retrievers, model.n_qpp)
    pred = model_predict(model, X)
    return {qid: {r: w for r, w in zip(retrievers, pred[i])} for i, qid in enumerate(all_qids)}

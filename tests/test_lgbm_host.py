"""Learned-fusion model reading and the LightGBM restatement (CPU).

The reference's NQ models are LightGBM boosters inside pickles; qppfuse.lgbm
decodes them without unpickling.  LightGBM itself is not installed, so the tree
walk is pinned by hand-built models with known answers (parity with the
library: unpinned).
"""
import gzip
import json
import math
from pathlib import Path

import numpy as np
import pytest

from oracle import lgbm_oracle

GOLD = Path(__file__).resolve().parent / "golden" / "lgbm"
REF_MODELS = Path("/root/reference/data/nq/models")

# two trees on 3 features; tree 0: f0 <= 0.5 ? (f1 <= 0.25 ? L0 : L1) : L2
# node 1 has missing type Zero + default left (decision_type 6), node 0 None (2);
# tree 1: a single leaf; tree 2: missing type NaN, default right (decision_type 8)
TOY = """tree
version=v4
num_class=1
num_tree_per_iteration=1
label_index=0
max_feature_idx=2
objective=regression
feature_names=a b c

Tree=0
num_leaves=3
num_cat=0
split_feature=0 1
split_gain=1 1
threshold=0.5 0.25
decision_type=2 6
left_child=1 -1
right_child=-3 -2
leaf_value=0.125 0.5 1.25
shrinkage=1

Tree=1
num_leaves=1
num_cat=0
leaf_value=0.0625
shrinkage=1

Tree=2
num_leaves=2
num_cat=0
split_feature=2
split_gain=1
threshold=1.5
decision_type=8
left_child=-1
right_child=-2
leaf_value=-0.25 2
shrinkage=0.05

end of trees
"""


def test_toy_model_known_answers():
    from qppfuse.lgbm import parse_lgbm_model
    b = parse_lgbm_model(TOY, best_iteration=0)
    assert len(b.used_trees) == 3
    cases = [
        ([0.4, 0.2, 1.0], 0.125 + 0.0625 - 0.25),
        ([0.4, 0.3, 2.0], 0.5 + 0.0625 + 2.0),
        ([0.6, 0.0, 1.5], 1.25 + 0.0625 - 0.25),           # <= threshold goes left
        ([0.4, 0.0, 5.0], 0.125 + 0.0625 + 2.0),           # Zero missing -> default left
        ([0.4, 1e-36, 0.0], 0.125 + 0.0625 - 0.25),        # |x| <= 1e-35 is "zero"
        ([float("nan"), 0.3, float("nan")], 0.5 + 0.0625 + 2.0),  # NaN: f0 read as 0; f2 default right
    ]
    for x, want in cases:
        got = lgbm_oracle.booster_predict(b, np.array([x]))[0]
        assert got == want, (x, got, want)
    # best_iteration limits the trees used
    assert len(parse_lgbm_model(TOY, best_iteration=2).used_trees) == 2


def test_weight_normalisation_is_the_references_numpy():
    rng = np.random.default_rng(0)
    raw = rng.standard_normal((500, 5))
    raw[:50] = -np.abs(raw[:50])  # all-negative rows -> sum 0 -> divide by 1
    w = lgbm_oracle.normalize_weights(raw)
    assert np.all(w[:50] == 0.0)
    ok = raw[50:].clip(0, None)
    sums = ok.sum(axis=1, keepdims=True)
    np.testing.assert_array_equal(w[50:], ok / np.where(sums == 0, 1.0, sums))


@pytest.mark.parametrize("corpus", ["nq", "hotpotqa", "scifact"])
@pytest.mark.parametrize("name", ["fusion_multioutput", "fusion_per_retriever"])
def test_fixtures_load_and_pack(name, corpus):
    from qppfuse import lgbm
    m = lgbm.load_fusion_model(GOLD / f"{corpus}_{name}.json.gz")
    assert m.retrievers == ["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade"]
    assert m.n_qpp == 13 and len(m.boosters) == 5
    p = lgbm.pack_model(m)
    assert p.n_features == 65 and p.tree_off[-1] == sum(len(b.used_trees) for b in m.boosters)
    assert set(np.unique(p.dtype).tolist()) <= {2}


@pytest.mark.skipif(not REF_MODELS.exists(), reason="reference checkout not present")
@pytest.mark.parametrize("corpus", ["nq", "hotpotqa", "scifact"])
@pytest.mark.parametrize("name", ["fusion_multioutput", "fusion_per_retriever"])
def test_static_pickle_reader_matches_fixture(name, corpus):
    """The committed fixture is exactly what the static decoder reads from the pickle."""
    from qppfuse import lgbm
    pkl = REF_MODELS.parent.parent / corpus / "models" / f"{name}.pkl"
    m = lgbm.load_fusion_model(pkl)
    with gzip.open(GOLD / f"{corpus}_{name}.json.gz", "rt") as fh:
        fx = json.load(fh)
    assert lgbm.model_to_fixture(m, lgbm.booster_texts(pkl)) == fx


def test_static_reader_never_resolves_classes(tmp_path):
    """A pickle naming a callable stays inert data (nothing imported or called)."""
    import pickle
    from qppfuse import lgbm
    path = tmp_path / "x.pkl"
    path.write_bytes(pickle.dumps({"a": [1, 2.5, "s"], "f": math.floor}, protocol=4))
    d = lgbm.read_pickle_static(path)
    assert d["a"] == [1, 2.5, "s"]
    assert isinstance(d["f"], lgbm.Opaque) and d["f"].name == "floor"

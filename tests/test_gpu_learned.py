"""Learned fusion on device vs the CPU restatement — needs an MI355X.

LightGBM inference (qf_gbdt_predict), the weight normalisation
(qf_learned_weights) and the fused lists / run file of learned_fusion are
compared bit for bit with oracle/lgbm_oracle.py + oracle/ref_port.py (the
reference's own pandas calls for the fusion step).
"""
from pathlib import Path

import numpy as np
import pandas as pd
import pytest
import torch

from oracle import lgbm_oracle, ref_port
from tests.test_lgbm_host import TOY

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden" / "lgbm"
NAMES = ["fusion_multioutput", "fusion_per_retriever"]
# every LightGBM model the reference holds (data/{nq,hotpotqa,scifact}/models): corpus_name
MODELS = [f"{c}_{n}" for c in ("nq", "hotpotqa", "scifact") for n in NAMES]


def _model(name):
    from qppfuse import lgbm
    if not name.startswith(("nq_", "hotpotqa_", "scifact_")):
        name = f"nq_{name}"
    return lgbm.load_fusion_model(GOLD / f"{name}.json.gz")


def _X(rng, n, f):
    X = rng.uniform(0, 1, (n, f))
    X[rng.random((n, f)) < 0.15] = 0.0          # zero features (missing qpp -> 0)
    m = rng.random((n, f)) < 0.05                # repeated values (one mask for both sides)
    X[m] = np.round(X[m].mean(), 6)
    return X


@pytest.mark.parametrize("name", MODELS)
def test_gbdt_predict_matches_restatement(gpu, name):
    from qppfuse import engine, lgbm
    m = _model(name)
    p = lgbm.pack_model(m)
    rng = np.random.default_rng(7)
    X = _X(rng, 600, p.n_features)
    # values exactly on thresholds take the left branch
    thr = p.threshold[:50]
    X[:50, p.feature[:50]] = thr
    got = engine.gbdt_predict(torch.from_numpy(X).to(gpu), p).cpu().numpy()
    want = np.column_stack([lgbm_oracle.booster_predict(b, X) for b in m.boosters])
    assert got.tobytes() == want.tobytes()


def test_gbdt_missing_types_and_single_leaf_trees(gpu):
    from qppfuse import engine, lgbm
    b = lgbm.parse_lgbm_model(TOY)
    m = lgbm.FusionModel("MultiOutputLGBM", ["a"], 3, [b])
    p = lgbm.pack_model(m)
    X = np.array([[0.4, 0.2, 1.0], [0.4, 0.3, 2.0], [0.6, 0.0, 1.5], [0.4, 0.0, 5.0],
                  [0.4, 1e-36, 0.0], [np.nan, 0.3, np.nan], [-0.0, -1e-40, 1.5]])
    got = engine.gbdt_predict(torch.from_numpy(X).to(gpu), p).cpu().numpy()[:, 0]
    want = lgbm_oracle.booster_predict(b, X)
    assert got.tobytes() == want.tobytes()


def test_gbdt_model_beyond_lds_walks_global_arrays(gpu):
    """A model too large for the kernel's LDS image (the NQ boosters' trees
    repeated 8 times: ~36 k nodes) takes the global-array walk — bit-exact too;
    and a row count that strides every wave over several rows."""
    import dataclasses
    from qppfuse import engine, lgbm
    m = _model("fusion_multioutput")
    big = [dataclasses.replace(b, trees=b.used_trees * 8, best_iteration=0) for b in m.boosters]
    mb = dataclasses.replace(m, boosters=big)
    p = lgbm.pack_model(mb)
    assert len(p.threshold) * 20 > 148 * 1024
    rng = np.random.default_rng(11)
    X = _X(rng, 97, p.n_features)
    got = engine.gbdt_predict(torch.from_numpy(X).to(gpu), p).cpu().numpy()
    want = np.column_stack([lgbm_oracle.booster_predict(b, X) for b in big])
    assert got.tobytes() == want.tobytes()
    small = lgbm.pack_model(m)
    X2 = _X(rng, 4200, small.n_features)  # > 256 workgroups x 16 waves: rows strided
    got2 = engine.gbdt_predict(torch.from_numpy(X2).to(gpu), small).cpu().numpy()
    want2 = np.column_stack([lgbm_oracle.booster_predict(b, X2) for b in m.boosters])
    assert got2.tobytes() == want2.tobytes()


@pytest.mark.parametrize("name", MODELS)
def test_learned_gbdt_weights_one_launch_equals_three(gpu, name):
    """qf_learned_gbdt_weights (features from the QPP micro-units, the walk and the
    weight normalisation in one launch) == qf_qpp_features + qf_gbdt_predict +
    qf_learned_weights bit for bit: predictions and weights, a model block whose
    retriever the batch lacks (-1), a run the model does not know (-1), zero and
    negative micro-units, a row count that is no multiple of the 16 rows in flight."""
    from qppfuse import engine, lgbm
    m = _model(name)
    p = lgbm.pack_model(m)
    rng = np.random.default_rng(13)
    Q, R = 1037, 6
    micro = rng.integers(-200_000, 1_200_000, (Q * R, 13)).astype(np.int64)
    micro[rng.random(micro.shape) < 0.2] = 0
    blocks = [3, 0, -1, 5, 1][:len(m.retrievers)]
    run_to_booster = [1, -1, 0, 3, 4, 2]
    mt = torch.from_numpy(micro).to(gpu)
    X = engine.qpp_features(mt, Q, R, blocks)
    pred3 = engine.gbdt_predict(X, p)
    w3 = engine.learned_weights(pred3, run_to_booster)
    w1, pred1 = engine.learned_gbdt_weights(mt, Q, R, blocks, p, run_to_booster, want_pred=True)
    assert torch.equal(pred1.view(torch.int64), pred3.view(torch.int64))
    assert torch.equal(w1.view(torch.int64), w3.view(torch.int64))
    assert torch.equal(engine.learned_gbdt_weights(mt, Q, R, blocks, p, run_to_booster)
                       .view(torch.int64), w3.view(torch.int64))


@pytest.mark.parametrize("mode", ["minmax", "zscore"])
def test_learned_gbdt_weights_from_raw_qpp(gpu, mode):
    """The one-launch learned weights fed the RAW predictors + column statistics
    (the normalisation folded in) == qpp_normalize's micro-units -> features ->
    GBDT -> weights, bit for bit; absent lists normalise to 0.0."""
    from qppfuse import engine, lgbm
    m = _model("fusion_multioutput")
    p = lgbm.pack_model(m)
    rng = np.random.default_rng(17)
    Q, R = 613, 5
    raw = rng.gamma(2, 3, (Q * R, 13))
    raw[:, 6] = 2.5                              # a constant column
    n = rng.integers(0, 4, Q * R)
    n[[1, 2, 40]] = 0                            # absent lists
    off = np.zeros(Q * R + 1, np.int64)
    off[1:] = np.cumsum(n)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    graw, goff = t(raw), t(off)
    stats = (engine.qpp_colminmax if mode == "minmax" else engine.qpp_colmeanstd)(graw, goff, R)
    micro = engine.qpp_normalize(graw, stats, goff, R, mode, 5, want_micro=True,
                                 want_weights=False)["micro"]
    blocks = list(range(len(m.retrievers)))
    rb = [0, 1, 2, 3, 4]
    want = engine.learned_gbdt_weights(micro, Q, R, blocks, p, rb)
    got = engine.learned_gbdt_weights(None, Q, R, blocks, p, rb, raw_qpp=graw, mm=stats,
                                      list_off=goff, mode=mode)
    assert torch.equal(got.view(torch.int64), want.view(torch.int64))


def test_learned_weights_match_numpy(gpu):
    from qppfuse import engine
    rng = np.random.default_rng(3)
    raw = rng.standard_normal((400, 5))
    raw[:40] = -np.abs(raw[:40])
    raw[40:60, 2] = 0.0
    raw[60:70] = -0.0
    rb = [4, -1, 0, 1, 2, 3]  # run order differs from model order; one unknown run
    got = engine.learned_weights(torch.from_numpy(raw).to(gpu), rb).cpu().numpy().reshape(400, 6)
    w = lgbm_oracle.normalize_weights(raw)
    want = np.column_stack([w[:, j] if j >= 0 else np.full(400, 1.0 / 5) for j in rb])
    assert got.tobytes() == want.tobytes()


def _runs(rng, qids, rankers, k, overlap=0.6, ties=False):
    frames = {}
    for r in rankers:
        rows = []
        for q in qids:
            pool = [f"d{q}_{i}" for i in range(2 * k)]
            docs = list(rng.choice(pool, size=k, replace=False)) if rng.random() < overlap else \
                [f"x{r}_{q}_{i}" for i in range(k)]
            sc = np.sort(rng.uniform(0, 1, k))[::-1]
            if ties:
                sc = np.round(sc * 4) / 4
            sc = np.round(sc, 6)
            rows += [(q, d, i + 1, float(s)) for i, (d, s) in enumerate(zip(docs, sc))]
        df = pd.DataFrame(rows, columns=["qid", "docno", "rank", "score"])
        df.insert(1, "iter", "Q0")
        df["runid"] = r
        frames[r] = df
    return frames


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("ties", [False, True])
def test_learned_fusion_matches_reference_pandas(gpu, name, ties, tmp_path, capsys):
    from qppfuse import fusion
    rng = np.random.default_rng(11 if ties else 12)
    model = _model(name)
    qids = [f"test{i}" for i in range(60)]
    rankers = ["Splade", "BM25", "BGE", "BM25_TCT", "BM25_MonoT5", "Extra"]  # listdir-like order
    runs = _runs(rng, qids, rankers, 40, ties=ties)
    qpp = {q: {r: [float(np.round(v, 6)) for v in rng.uniform(0, 1, 13)]
               for r in model.retrievers if rng.random() < 0.9} for q in qids[:-3]}
    got = fusion.learned_fusion(runs, qpp, str(GOLD / f"{name}.json.gz"))
    wd = lgbm_oracle.weights_dict(runs, qpp, model)
    want = ref_port.learned_fusion_from_weights(runs, wd, len(model.retrievers))
    assert list(got.keys()) == sorted(want.keys())
    for q in want:
        assert got[q] == want[q], q
    p = tmp_path / "learned.res"
    fusion.write_runfile(got, str(p), "learned")
    assert p.read_text() == ref_port.runfile_text(want, "learned")


@pytest.mark.parametrize("k,ties", [(1000, False), (1000, True), (700, True)])
def test_learned_fusion_large_lists_join_and_sort_in_one_kernel(gpu, k, ties):
    """5 runs x top-k (C5's shape: 1,025-5,120 entries per query, micro-unit
    scores) take join_learned_kernel — the join, the Kahan sums and the docid-tie
    bucket sort in one workgroup, unions up to 4,608 (SURVEY §8(d)'s ~4,030) — bit
    for bit the reference's pandas calls; larger unions take the fallback pass."""
    from qppfuse import fusion
    rng = np.random.default_rng(k + ties)
    model = _model("fusion_multioutput")
    qids = [f"test{i}" for i in range(24)]
    runs = _runs(rng, qids, ["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade"], k, ties=ties)
    qpp = {q: {r: [float(np.round(v, 6)) for v in rng.uniform(0, 1, 13)]
               for r in model.retrievers} for q in qids}
    got = fusion.learned_fusion(runs, qpp, str(GOLD / "nq_fusion_multioutput.json.gz"))
    wd = lgbm_oracle.weights_dict(runs, qpp, model)
    want = ref_port.learned_fusion_from_weights(runs, wd, len(model.retrievers))
    assert list(got.keys()) == sorted(want.keys())
    for q in want:
        assert got[q] == want[q], q
    if k == 1000:  # unions on both sides of kJsUMax and of kLearnedUMax
        us = [len(want[q]) for q in qids]
        assert any(u <= 3072 for u in us) and any(3072 < u <= 4608 for u in us)
        assert any(u > 4608 for u in us)
    for q in qids[:3]:  # and the ranked order write_runfile takes
        ids, sc = got.arrays(q)
        w = sorted(want[q], key=lambda x: x[1], reverse=True)
        assert [s for _, s in w] == sc.tolist()
        assert [d for d, _ in w] == got._docnos[ids].tolist()  # ties in docno order


@pytest.mark.parametrize("dups", [False, True])
def test_learned_fusion_18_runs_and_duplicates(gpu, dups):
    """18 runs (5 the model knows + 13 it does not: weight 1/n_retrievers,
    src/fusion.py:435) through the workspace join, and docnos repeated inside one
    list (the groupby adds every row, src/fusion.py:440-441): == the reference's
    pandas calls (oracle/ref_port.py) bit for bit."""
    from qppfuse import fusion
    rng = np.random.default_rng(18 + dups)
    model = _model("fusion_multioutput")
    qids = [f"test{i}" for i in range(25)]
    rankers = list(model.retrievers) + [f"X{i:02d}" for i in range(13)]
    runs = _runs(rng, qids, rankers, 30)
    if dups:
        for r in rankers[::3]:
            df = runs[r]
            extra = df.sample(frac=0.2, random_state=int(rng.integers(1 << 30))).copy()
            extra["score"] = np.round(rng.uniform(0, 1, len(extra)), 6)
            runs[r] = pd.concat([df, extra], ignore_index=True)
    qpp = {q: {r: [float(np.round(v, 6)) for v in rng.uniform(0, 1, 13)]
               for r in model.retrievers} for q in qids}
    got = fusion.learned_fusion(runs, qpp, str(GOLD / "nq_fusion_multioutput.json.gz"))
    wd = lgbm_oracle.weights_dict(runs, qpp, model)
    want = ref_port.learned_fusion_from_weights(runs, wd, len(model.retrievers))
    assert list(got.keys()) == sorted(want.keys())
    for q in want:
        assert got[q] == want[q], q


# ---- FusionMLP (src/models/mlp_model.py:254-274 through src/fusion.py:387-448) ----

MLP_GOLD = Path(__file__).resolve().parent / "golden" / "mlp"
MLP_DS = ["nq", "hotpotqa", "scifact"]


def _mlp(ds):
    from qppfuse import mlp
    return mlp.load_mlp_fixture(MLP_GOLD / f"{ds}_fusion_mlp.json.gz")


def _mlp_want(m, X, rb):
    from oracle import mlp_oracle
    w = mlp_oracle.predict(m.layers, m.retrievers, m.n_qpp, m.qpp_indices, X)
    n = len(m.retrievers)
    return np.column_stack([w[:, j].astype(np.float64) if j >= 0 else np.full(len(X), 1.0 / n)
                            for j in rb])


@pytest.mark.parametrize("ds", MLP_DS)
def test_mlp_weights_match_restatement(gpu, ds):
    """qf_mlp_weights == the float32 restatement bit for bit (zeros, constant rows,
    out-of-range features that saturate the softmax)."""
    from qppfuse import engine
    m = _mlp(ds)
    rng = np.random.default_rng(40)
    X = _X(rng, 700, m.n_qpp * len(m.retrievers))
    X[:20] *= 1e3
    X[20:40] = -X[20:40]
    X[40] = 0.0
    rb = [4, -1, 0, 1, 2, 3]
    got = engine.mlp_weights(torch.from_numpy(X).to(gpu), m, rb).cpu().numpy().reshape(700, 6)
    assert got.tobytes() == _mlp_want(m, X, rb).tobytes()


def test_mlp_weights_wide_model_all_features(gpu):
    """Every QPP column as input (no _filter_features), layers wider than a wave
    (128 and 96 lanes' worth of outputs), six outputs: == the restatement."""
    from qppfuse import engine, mlp
    rng = np.random.default_rng(41)
    rets = [f"r{i}" for i in range(6)]
    widths = [6 * 13, 128, 96, 6]
    layers = [((rng.standard_normal((o, i)) / np.sqrt(i)).astype(np.float32),
               (0.1 * rng.standard_normal(o)).astype(np.float32))
              for i, o in zip(widths[:-1], widths[1:])]
    m = mlp.MLPModel(rets, 13, list(range(13)), layers)
    m.validate()
    X = _X(rng, 300, 6 * 13)
    rb = list(range(6))
    got = engine.mlp_weights(torch.from_numpy(X).to(gpu), m, rb).cpu().numpy().reshape(300, 6)
    assert got.tobytes() == _mlp_want(m, X, rb).tobytes()


@pytest.mark.parametrize("ds", MLP_DS)
def test_mlp_weights_vs_reference_predict(gpu, ds):
    """Against the reference's own FusionMLP.predict (torch CPU): float32 rounding."""
    from qppfuse import engine
    from tests.test_mlp_host import W_ULPS, _arr, _gold, ulp_diff
    e = _gold()[ds]
    m = _mlp(ds)
    X = _arr(e["X"], "<f8", (e["n_rows"], e["cols"]))
    want = _arr(e["predict"], "<f4", (e["n_rows"], -1))
    got = engine.mlp_weights(torch.from_numpy(X.copy()).to(gpu), m,
                             list(range(5))).cpu().numpy().reshape(e["n_rows"], 5)
    assert np.array_equal(got.astype(np.float32).astype(np.float64), got)  # float32 values
    assert ulp_diff(got, want).max() <= W_ULPS


@pytest.mark.parametrize("case", [0, 1])
def test_mlp_learned_fusion_vs_reference(gpu, case, tmp_path):
    """learned_fusion with the NQ FusionMLP: bit for bit the reference's pandas calls
    on the restatement's weights (float32 products and a float32 groupby sum for the
    known rankers; a float64 column once a ranker is unknown), and within float32
    rounding of the reference's own learned_fusion output."""
    from oracle import mlp_oracle
    from qppfuse import fusion
    from tests.test_mlp_host import _frames, _gold, assert_fused_close
    c = _gold()["nq"]["fusion"][case]
    m = _mlp("nq")
    runs = _frames(c["runs"])
    got = fusion.learned_fusion(runs, c["qpp"], str(MLP_GOLD / "nq_fusion_mlp.json.gz"))
    wd = mlp_oracle.weights_dict(runs, c["qpp"], m)
    want = ref_port.learned_fusion_from_weights(runs, wd, len(m.retrievers))
    assert list(got.keys()) == sorted(want.keys())
    for q in want:
        assert got[q] == want[q], q
    assert_fused_close(got, c["fused"])
    p = tmp_path / "learned_mlp.res"
    fusion.write_runfile(got, str(p), "learned_mlp")
    assert p.read_text() == ref_port.runfile_text(want, "learned_mlp")


@pytest.mark.parametrize("extra", [0, 13])
def test_mlp_learned_fusion_duplicates(gpu, extra):
    """Docnos repeated inside a list (virtual runs: every row adds) with only known
    rankers (float32 column) and with 13 unknown rankers (18 runs, workspace join,
    float64 column): == the reference's pandas calls bit for bit."""
    from oracle import mlp_oracle
    from qppfuse import fusion
    rng = np.random.default_rng(50 + extra)
    m = _mlp("scifact")
    qids = [f"test{i}" for i in range(25)]
    rankers = list(m.retrievers) + [f"X{i:02d}" for i in range(extra)]
    runs = _runs(rng, qids, rankers, 30)
    for r in rankers[::2]:
        df = runs[r]
        dup = df.sample(frac=0.2, random_state=int(rng.integers(1 << 30))).copy()
        dup["score"] = np.round(rng.uniform(0, 1, len(dup)), 6)
        runs[r] = pd.concat([df, dup], ignore_index=True)
    qpp = {q: {r: [float(np.round(v, 6)) for v in rng.uniform(0, 1, 13)]
               for r in m.retrievers} for q in qids}
    got = fusion.learned_fusion(runs, qpp, str(MLP_GOLD / "scifact_fusion_mlp.json.gz"))
    wd = mlp_oracle.weights_dict(runs, qpp, m)
    want = ref_port.learned_fusion_from_weights(runs, wd, len(m.retrievers))
    assert list(got.keys()) == sorted(want.keys())
    for q in want:
        assert got[q] == want[q], q

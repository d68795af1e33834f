"""FusionMLP learned fusion on the host: the static pickle decoder, the fixtures,
and the CPU restatement (oracle/mlp_oracle.py) against the reference's own
FusionMLP.predict / learned_fusion outputs (tests/golden/make_mlp_golden.py).

The restatement fixes one float32 operation order (the device's); torch's CPU
kernels round in another, so against the reference the bar is float32 rounding:
weights within 8 ulp (measured: <= 5), fused scores within 1e-6 relative.  The
device is held to the restatement bit for bit (tests/test_gpu_learned.py).
"""
import base64
import gzip
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import mlp_oracle, ref_port

GOLD = Path(__file__).resolve().parent / "golden" / "mlp"
REF = Path("/root/reference")
DATASETS = ["nq", "hotpotqa", "scifact"]
W_ULPS = 8
S_RTOL = 1e-6


def _gold():
    with gzip.open(GOLD / "reference_mlp.json.gz", "rt") as fh:
        return json.load(fh)


def _arr(s, dt, shape):
    return np.frombuffer(base64.b64decode(s), dt).reshape(shape)


def _fixture(ds):
    from qppfuse import mlp
    return mlp.load_mlp_fixture(GOLD / f"{ds}_fusion_mlp.json.gz")


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)


@pytest.mark.parametrize("ds", DATASETS)
def test_fixture_layout(ds):
    m = _fixture(ds)
    assert m.retrievers == ["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade"]
    assert (m.n_qpp, m.qpp_indices, m.widths()) == (13, [5], [5, 32, 16, 5])
    assert list(m.input_columns()) == [5, 18, 31, 44, 57]  # RSD of each retriever
    assert m.flat_params().dtype == np.float32
    assert m.flat_params().size == 5 * 32 + 32 + 32 * 16 + 16 + 16 * 5 + 5


@pytest.mark.skipif(not REF.exists(), reason="needs /root/reference (build container)")
@pytest.mark.parametrize("ds", DATASETS)
def test_static_decode_of_reference_pickle(ds):
    """The reference's fusion_mlp.pkl decoded as data equals the committed fixture,
    and its two copies of the weights (the object's Sequential and model_state)
    agree element for element."""
    from qppfuse import mlp
    from qppfuse.lgbm import read_pickle_static
    path = REF / f"data/{ds}/models/fusion_mlp.pkl"
    m = mlp.load_mlp_model(path)
    fx = _fixture(ds)
    for (W, b), (W2, b2) in zip(m.layers, fx.layers):
        assert W.tobytes() == W2.tobytes() and b.tobytes() == b2.tobytes()
    top = read_pickle_static(path)
    kv = top["model_state"].items
    seq = top["model"].state["model"].state["_modules"]
    for i in range(0, len(kv), 2):
        li, name = kv[i].split(".")
        a = mlp.decode_tensor(seq[li].state["_parameters"][name])
        assert a.tobytes() == mlp.decode_tensor(kv[i + 1]).tobytes(), kv[i]


def test_decode_storage_rejects_other_streams():
    import pickle
    from qppfuse import mlp
    with pytest.raises(ValueError):
        mlp.decode_storage(pickle.dumps(1) * 5)


def test_mlp_model_kind(tmp_path):
    from qppfuse import mlp
    assert mlp.model_kind(GOLD / "nq_fusion_mlp.json.gz") == "FusionMLP"
    lg = Path(__file__).resolve().parent / "golden" / "lgbm" / "nq_fusion_multioutput.json.gz"
    assert mlp.model_kind(lg) is None


@pytest.mark.parametrize("ds", DATASETS)
def test_oracle_predict_vs_reference(ds):
    e = _gold()[ds]
    m = _fixture(ds)
    X = _arr(e["X"], "<f8", (e["n_rows"], e["cols"]))
    want = _arr(e["predict"], "<f4", (e["n_rows"], -1))
    got = mlp_oracle.predict(m.layers, m.retrievers, m.n_qpp, m.qpp_indices, X)
    assert got.dtype == np.float32
    assert ulp_diff(got, want).max() <= W_ULPS
    np.testing.assert_allclose(got.sum(axis=1), 1.0, rtol=1e-6)


def _frames(runs):
    import pandas as pd
    out = {}
    for r, rows in runs.items():
        df = pd.DataFrame(rows, columns=["qid", "docno", "rank", "score"])
        df.insert(1, "iter", "Q0")
        df["runid"] = r
        df["qid"] = df["qid"].astype(str)
        out[r] = df
    return out


def assert_fused_close(got, gold_fused):
    assert sorted(got) == sorted(gold_fused)
    for q, lst in gold_fused.items():
        g = got[q]
        assert [d for d, _ in g] == [d for d, _ in lst], q
        a = np.array([float(s) for _, s in g])
        b = np.array([float.fromhex(s) for _, s in lst])
        np.testing.assert_allclose(a, b, rtol=S_RTOL, atol=0, err_msg=q)


@pytest.mark.parametrize("case", [0, 1])
def test_oracle_learned_fusion_vs_reference(case):
    """The restatement's weights through the reference's own pandas calls
    (ref_port) reproduce the reference's learned_fusion: float32 scores for the
    five known rankers, float64 once a ranker is unknown."""
    c = _gold()["nq"]["fusion"][case]
    m = _fixture("nq")
    runs = _frames(c["runs"])
    wd = mlp_oracle.weights_dict(runs, c["qpp"], m)
    got = ref_port.learned_fusion_from_weights(runs, wd, len(m.retrievers))
    assert_fused_close(got, c["fused"])
    vals = [float(s) for lst in got.values() for _, s in lst]
    f32 = all(float(np.float32(v)) == v for v in vals)
    assert f32 == (not c["extra"])


@pytest.mark.parametrize("offset,size,stride", [
    (0, (3, 4), (4, 1)),      # the whole storage: accepted
    (0, (3, 5), (4, 1)),      # one element past the end
    (13, (1,), (1,)),         # offset past the storage
    (-1, (2,), (1,)),         # negative offset
    (0, (2, 2), (-1, 1)),     # negative stride
    (0, (4,), (1, 1)),        # rank mismatch
    (11, (2,), (1,)),         # starts inside, runs past
    (0, (0, 99), (99, 1)),    # an empty view: nothing read
])
def test_decode_tensor_checks_geometry(monkeypatch, offset, size, stride):
    """A tampered size / stride / offset in the pickle must not reach as_strided
    (an out-of-bounds read): ValueError instead."""
    from qppfuse import mlp
    from qppfuse.lgbm import Opaque
    monkeypatch.setattr(mlp, "decode_storage", lambda blob: np.arange(12, dtype=np.float32))
    t = Opaque("torch._utils", "_rebuild_tensor_v2",
               (Opaque("torch.storage", "_load_from_bytes", (b"",)), offset, size, stride))
    ok = (offset, size, stride) in [(0, (3, 4), (4, 1)), (0, (0, 99), (99, 1))]
    if ok:
        a = mlp.decode_tensor(t)
        assert a.shape == size
        if a.size:
            assert a.tobytes() == np.arange(12, dtype=np.float32).reshape(3, 4).tobytes()
    else:
        with pytest.raises(ValueError):
            mlp.decode_tensor(t)

#!/usr/bin/env python3
"""Golden fixtures for FusionMLP learned fusion, from the REFERENCE itself.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/make_mlp_golden.py
1. Decodes the reference's three data/<ds>/models/fusion_mlp.pkl statically
   (qppfuse.mlp: nothing unpickled) into tests/golden/mlp/<ds>_fusion_mlp.json.gz.
2. Builds the reference's own FusionMLP class (src/models/mlp_model.py, imported by
   file path; lightgbm and ir_measures are absent, so src/models/__init__.py and
   src/evaluation/ir_evaluator.py are bypassed / stubbed) on the CPU, loads those
   decoded weights into it with load_state_dict, and records its predict(X) on a
   synthetic feature matrix.
3. Runs the reference's learned_fusion (src/fusion.py:387-448) with that model on
   synthetic runs: once with the five retrievers the model knows (float32 weights,
   a float32 groupby column under numpy 2) and once with an extra ranker it does
   not know (1.0 / n_retrievers: a float64 column).  learned_fusion's
   pickle.load is replaced by a function returning the in-memory model dict, so no
   pickle is read at all.
Outputs are data only: inputs, weights (float32, base64) and fused lists (float.hex).
"""
from __future__ import annotations

import base64
import gzip
import importlib.util
import io
import json
import random
import sys
import types
from contextlib import redirect_stdout
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "qpp-fusion-rag_amd"))
sys.path.insert(0, str(HERE))

import make_golden as mg  # noqa: E402
from qppfuse import mlp  # noqa: E402

OUT = HERE / "mlp"
DATASETS = ["nq", "hotpotqa", "scifact"]


def b64(a, dt):
    return base64.b64encode(np.ascontiguousarray(a, dt).tobytes()).decode()


def load_mlp_module():
    mods = mg.load_reference()
    ev = types.ModuleType("src.evaluation")
    ev.__path__ = []
    sys.modules["src.evaluation"] = ev
    ire = types.ModuleType("src.evaluation.ir_evaluator")
    ire.compute_ndcg = None  # base.py:160 re-exports it; unused here
    sys.modules["src.evaluation.ir_evaluator"] = ire
    pkg = types.ModuleType("src.models")
    pkg.__path__ = [str(mg.REF / "src/models")]
    sys.modules["src.models"] = pkg

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    load("src.models.base", mg.REF / "src/models/base.py")
    mods["mlp_model"] = load("src.models.mlp_model", mg.REF / "src/models/mlp_model.py")
    return mods


def reference_model(mods, m: mlp.MLPModel):
    import torch
    with redirect_stdout(io.StringIO()):
        fm = mods["mlp_model"].FusionMLP(m.retrievers, n_qpp=m.n_qpp, qpp_indices=m.qpp_indices,
                                         hidden_sizes=m.widths()[1:-1], device="cpu")
    sd = {}
    lin = [k for k, v in fm.model.named_children() if isinstance(v, torch.nn.Linear)]
    for name, (W, b) in zip(lin, m.layers):
        sd[f"{name}.weight"] = torch.from_numpy(np.array(W))
        sd[f"{name}.bias"] = torch.from_numpy(np.array(b))
    fm.model.load_state_dict(sd)
    fm.model.eval()
    fm.is_trained = True
    return fm


def synth_X(rng: np.random.Generator, n: int, cols: int) -> np.ndarray:
    X = np.round(rng.uniform(0, 1, (n, cols)), 6)
    X[rng.random((n, cols)) < 0.1] = 0.0  # missing QPP entries -> 0
    X[0] = 0.0  # constant rows
    X[1] = 1.0
    X[2] = 0.5
    X[3] = 1e-6
    return X


def fusion_case(mods, fm, m, seed, extra):
    rng = random.Random(seed)
    rankers = list(m.retrievers) + (["Extra"] if extra else [])
    rng.shuffle(rankers)  # listdir-like order differs from the model's
    pool = [f"doc{i}" for i in range(120)]
    qids, runs = mg.make_case(rng, 24, rankers, (10, 30), pool, p_skip=0.05)
    qpp = mg.make_qpp(rng, qids[:-2], m.retrievers)  # two queries without QPP rows
    frames = mg.to_frames(runs)
    data = {"model": fm, "model_type": "FusionMLP", "retrievers": m.retrievers,
            "n_qpp": m.n_qpp}
    fus = mods["fusion"]
    saved = fus.pickle
    fus.pickle = types.SimpleNamespace(load=lambda f: data)
    try:
        with redirect_stdout(io.StringIO()):  # model_path is only opened, never read
            got = fus.learned_fusion(frames, qpp, __file__)
    finally:
        fus.pickle = saved
    types_seen = sorted({type(s).__name__ for lst in got.values() for _, s in lst})
    return {"runs": runs, "qpp": qpp, "extra": extra, "score_types": types_seen,
            "fused": mg.enc_fused(got)}


def main():
    OUT.mkdir(exist_ok=True)
    mods = load_mlp_module()
    out = {}
    for i, ds in enumerate(DATASETS):
        m = mlp.load_mlp_model(mg.REF / f"data/{ds}/models/fusion_mlp.pkl")
        with gzip.open(OUT / f"{ds}_fusion_mlp.json.gz", "wt") as fh:
            json.dump(mlp.mlp_to_fixture(m), fh)
        fm = reference_model(mods, m)
        nprng = np.random.default_rng(100 + i)
        X = synth_X(nprng, 256, m.n_qpp * len(m.retrievers))
        W = fm.predict(X)
        assert W.dtype == np.float32
        entry = {"X": b64(X, "<f8"), "n_rows": int(X.shape[0]), "cols": int(X.shape[1]),
                 "predict": b64(W, "<f4")}
        if ds == "nq":
            entry["fusion"] = [fusion_case(mods, fm, m, 7, False),
                               fusion_case(mods, fm, m, 8, True)]
        out[ds] = entry
    with gzip.open(OUT / "reference_mlp.json.gz", "wt") as fh:
        json.dump(out, fh, sort_keys=True)
    print("FusionMLP fixtures written to", OUT)


if __name__ == "__main__":
    main()

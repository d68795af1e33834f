"""Extract the reference's learned-fusion LightGBM models into JSON fixtures.

Reads /root/reference/data/{nq,hotpotqa,scifact}/models/fusion_{multioutput,
per_retriever}.pkl (every LightGBM model the reference holds) with
qppfuse.lgbm's static pickle decoder (nothing in the files is imported or
executed) and writes tests/golden/lgbm/<corpus>_<name>.json.gz: model type, retrievers,
n_qpp and every booster's LightGBM model text + best_iteration — the data the
pickles hold, so the GPU tests can run where the reference is absent.
"""
import gzip
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "qpp-fusion-rag_amd")]
from qppfuse import lgbm  # noqa: E402

DATA = Path("/root/reference/data")
OUT = Path(__file__).resolve().parent / "lgbm"
CORPORA = ("nq", "hotpotqa", "scifact")

if __name__ == "__main__":
    OUT.mkdir(exist_ok=True)
    for corpus in CORPORA:
        for name in ("fusion_multioutput", "fusion_per_retriever"):
            pkl = DATA / corpus / "models" / f"{name}.pkl"
            model = lgbm.load_fusion_model(pkl)
            fx = lgbm.model_to_fixture(model, lgbm.booster_texts(pkl))
            with gzip.open(OUT / f"{corpus}_{name}.json.gz", "wt") as fh:
                json.dump(fx, fh)
            print(corpus, name, model.model_type, model.retrievers,
                  [len(b.used_trees) for b in model.boosters])

"""The reference's driver sequence file to file on qppfuse — needs an MI355X.

scripts/05_fusion.py:56-152 (run_all_methods: three unweighted runs, the W-* runs named
by qpp_model.lower() with their tags, the learned loop over the per_retriever /
multioutput / mlp models) and scripts/06_eval_fusion.py:52-140 (every fused run
evaluated, comparison_results.json), replayed by tests/driver_replay.py on SURVEY §8(d)
runs with the real NQ qrels; every written file's rows of a 64-query sample equal the CPU
reference path's (oracle/ref_port.py: the reference's per-row algorithms; the LightGBM /
FusionMLP restatements) byte for byte, and the evaluation equals the C trec_eval
restatement.  tools/e2e.py --replay runs the same at C2 scale (profiles/r05_e2e.json)."""
import gzip
import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def test_run_all_methods_then_eval_match_the_cpu_reference(gpu, tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    sys.path.insert(0, str(ROOT / "tests"))
    import driver_replay as dr
    import e2e
    Q = 120
    runs_dir = tmp_path / "runs"
    runs_dir.mkdir()
    e2e.generate(runs_dir, Q, 5, 1000)
    fused_dir = tmp_path / "fused"
    fused_dir.mkdir()
    results = dr.run_all_methods(runs_dir, runs_dir / "qpp", fused_dir, qpp_model="RSD",
                                 model_files=e2e.MODEL_FILES)
    assert sorted(p.name for p in results.values()) == sorted(
        ["combsum.res", "combmnz.res", "rrf.res", "wcombsum_rsd.res", "wcombmnz_rsd.res",
         "wrrf_rsd.res", "learned_per_retriever.res", "learned_multioutput.res",
         "learned_mlp.res"])
    for key, p in results.items():  # tags as the script writes them
        tag = open(p).readline().split()[5]
        assert tag == {"wcombsum": "wcombsum-rsd", "wcombmnz": "wcombmnz-rsd",
                       "wrrf": "wrrf-rsd"}.get(key, key.replace("_", "-", 1)
                                                if key.startswith("learned") else key), key
    sample = [f"test{q}" for q in sorted(np.random.default_rng(1).choice(Q, 64, replace=False))]
    ok = dr.check_sample(runs_dir, runs_dir / "qpp", results, sample,
                         model_files=e2e.MODEL_FILES)
    assert all(ok.values()), ok
    qrels = tmp_path / "test.tsv"
    qrels.write_bytes(gzip.decompress((ROOT / "tests" / "golden" / "nq_qrels_test.tsv.gz")
                                      .read_bytes()))
    evals = dr.evaluate_fused_runs(fused_dir, qrels, tmp_path)
    on_disk = json.loads((tmp_path / "comparison_results.json").read_text())
    assert [r["method"] for r in on_disk] == [r["method"] for r in evals]
    assert len(evals) == 9 and all(r["n_queries"] == Q for r in evals)
    assert dr.check_eval(fused_dir, qrels, evals)

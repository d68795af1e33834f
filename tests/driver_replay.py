"""The reference's fusion and evaluation drivers replayed on qppfuse (test / tool helper).

`run_all_methods` is scripts/05_fusion.py:56-152 statement for statement with the
drop-in's names (load_runs, combsum, combmnz, rrf, load_qpp_scores, get_qpp_index,
weighted_*, learned_fusion, write_runfile): the same files (combsum.res, ...,
wcombsum_<qpp_model.lower()>.res, learned_<model>.res), tags and order, the learned
loop over models/fusion_{per_retriever,multioutput,mlp}.pkl.  `evaluate_fused_runs` is
scripts/06_eval_fusion.py:52-140 (load_qrels, every fused/*.res through load_run_file and
IREvaluator with the config's first six metrics, sorted by nDCG@10, written to
comparison_results.json).

`check_sample` recomputes the rows of a sample of queries of every written file on the
CPU reference path (oracle/ref_port.py: the reference's own per-row algorithms, the
LightGBM / FusionMLP restatements for the learned files) from the same `.norm.res` /
`.qpp` text, and compares them byte for byte; `check_eval` recomputes the evaluation with
the C trec_eval restatement (oracle/eval_oracle.c).  Used by tests/test_gpu_driver.py and
tools/e2e.py --replay."""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path
from typing import Dict, Iterable, List, Optional

import numpy as np

LEARNED = ["per_retriever", "multioutput", "mlp"]


def run_all_methods(runs_dir: Path, qpp_dir: Path, fused_dir: Path, qpp_model: str = None,
                    rrf_k: int = None, model_files: Optional[Dict[str, Path]] = None):
    """scripts/05_fusion.py:56-152 on qppfuse.  model_files: the learned models by name
    (default: fused_dir.parent / "models" / f"fusion_{name}.pkl", as the script; a
    fixture path may stand in for a pickle)."""
    from qppfuse.config import config
    from qppfuse.fusion import (combmnz, combsum, get_qpp_index, learned_fusion, load_qpp_scores,
                                load_runs, rrf, weighted_combmnz, weighted_combsum,
                                weighted_rrf, write_runfile)
    qpp_model = qpp_model or config.qpp.default_method
    rrf_k = rrf_k if rrf_k is not None else config.fusion.rrf_k
    results = {}
    runs = load_runs(str(runs_dir), use_normalized=True)
    fused = combsum(runs)
    write_runfile(fused, str(fused_dir / "combsum.res"), "combsum")
    results["combsum"] = fused_dir / "combsum.res"
    fused = combmnz(runs)
    write_runfile(fused, str(fused_dir / "combmnz.res"), "combmnz")
    results["combmnz"] = fused_dir / "combmnz.res"
    fused = rrf(runs, k=rrf_k)
    write_runfile(fused, str(fused_dir / "rrf.res"), "rrf")
    results["rrf"] = fused_dir / "rrf.res"
    if qpp_dir.exists():
        qpp_data = load_qpp_scores(str(qpp_dir))
        qpp_index = get_qpp_index(qpp_model)
        m = qpp_model.lower()
        fused = weighted_combsum(runs, qpp_data, qpp_index)
        write_runfile(fused, str(fused_dir / f"wcombsum_{m}.res"), f"wcombsum-{m}")
        results["wcombsum"] = fused_dir / f"wcombsum_{m}.res"
        fused = weighted_combmnz(runs, qpp_data, qpp_index)
        write_runfile(fused, str(fused_dir / f"wcombmnz_{m}.res"), f"wcombmnz-{m}")
        results["wcombmnz"] = fused_dir / f"wcombmnz_{m}.res"
        fused = weighted_rrf(runs, qpp_data, qpp_index, k=rrf_k)
        write_runfile(fused, str(fused_dir / f"wrrf_{m}.res"), f"wrrf-{m}")
        results["wrrf"] = fused_dir / f"wrrf_{m}.res"
        models_dir = fused_dir.parent / "models"
        for name in LEARNED:
            f = (model_files or {}).get(name, models_dir / f"fusion_{name}.pkl")
            if Path(f).exists():
                fused = learned_fusion(runs, qpp_data, str(f))
                write_runfile(fused, str(fused_dir / f"learned_{name}.res"), f"learned-{name}")
                results[f"learned_{name}"] = fused_dir / f"learned_{name}.res"
    return results


def evaluate_fused_runs(fused_dir: Path, qrels_path: Path, output_dir: Path):
    """scripts/06_eval_fusion.py:52-140 on qppfuse (without its printed table)."""
    from qppfuse.config import config
    from qppfuse.data_utils import load_qrels, load_run_file as _load_run
    from qppfuse.evaluation import IREvaluator

    def load_run_file(run_path):  # scripts/06_eval_fusion.py:42-49
        return {qid: sorted([(d, s) for d, s, r in docs], key=lambda x: -x[1])
                for qid, docs in _load_run(run_path).items()}

    qrels = load_qrels(qrels_path)
    res_files = sorted(fused_dir.glob("*.res"))
    evaluator = IREvaluator(metrics=config.evaluation.ir_metrics[:6])
    results = []
    for res_file in res_files:
        method_name = res_file.stem
        print(f"[eval] {method_name}", file=sys.stderr, flush=True)  # (the script prints too)
        run = load_run_file(res_file)
        if method_name.startswith("learned"):
            method_type = "learned"
        elif method_name.startswith("w"):
            method_type = "qpp-weighted"
        else:
            method_type = "unweighted"
        metrics = evaluator.evaluate(run, qrels, per_query=False)
        metrics["n_queries"] = len([q for q in run.keys() if q in qrels])
        results.append({"method": method_name, "type": method_type, **metrics})
    results.sort(key=lambda x: -x.get("nDCG@10", 0))
    with open(output_dir / "comparison_results.json", "w") as f:
        json.dump(results, f, indent=2)
    return results


# ---- the CPU reference path on a sample ----------------------------------------------------

def _frames(runs_dir: Path, qids: Iterable[str]):
    """The sample's rows of every *.norm.res, as the reference's load_runs frames (file
    order, os.listdir order of the rankers)."""
    import pandas as pd
    keep = set(qids)
    frames = {}
    for f in os.listdir(runs_dir):  # src/fusion.py:60 — listdir order
        if not f.endswith(".norm.res"):
            continue
        rows = [ln.split() for ln in open(runs_dir / f) if ln.split(None, 1)[0] in keep]
        frames[f.replace(".norm.res", "")] = pd.DataFrame(
            {"qid": [r[0] for r in rows], "iter": [r[1] for r in rows],
             "docno": [r[2] for r in rows], "rank": [int(r[3]) for r in rows],
             "score": [float(r[4]) for r in rows], "runid": [r[5] for r in rows]})
    return frames


def _qpp_text(qpp_dir: Path, qids: Iterable[str]):
    """load_qpp_scores of the sample (src/data_utils.py:262-293): {qid: {ranker: [13]}}."""
    keep = set(qids)
    out = {}
    for f in sorted(os.listdir(qpp_dir)):
        if not f.endswith(".mmnorm.qpp"):
            continue
        ranker = f.replace(".res.mmnorm.qpp", "")
        for ln in open(qpp_dir / f):
            parts = ln.rstrip("\n").split("\t")
            if parts[0] in keep:
                out.setdefault(parts[0], {})[ranker] = [float(x) for x in parts[1:]]
    return out


def _file_rows(path: Path, qids: Iterable[str]) -> str:
    keep = set(qids)
    return "".join(ln for ln in open(path) if ln.split(None, 1)[0] in keep)


def check_sample(runs_dir: Path, qpp_dir: Path, results: Dict[str, Path], qids: List[str],
                 qpp_model: str = "RSD", rrf_k: int = 60,
                 model_files: Optional[Dict[str, Path]] = None) -> Dict[str, bool]:
    """Every written file's rows of `qids` == the CPU reference path's rows, byte for byte."""
    from oracle import lgbm_oracle, mlp_oracle, ref_port
    from qppfuse import lgbm, mlp
    from qppfuse.config import get_qpp_index
    frames = _frames(runs_dir, qids)
    qpp = _qpp_text(qpp_dir, qids)
    qidx = get_qpp_index(qpp_model)
    m = qpp_model.lower()
    tags = {"combsum": "combsum", "combmnz": "combmnz", "rrf": "rrf",
            "wcombsum": f"wcombsum-{m}", "wcombmnz": f"wcombmnz-{m}", "wrrf": f"wrrf-{m}"}
    ok = {}
    for key, path in results.items():
        print(f"[check] {path.name}", file=sys.stderr, flush=True)
        if key in tags:
            fused = ref_port.fuse(frames, key, qpp, qidx, rrf_k)
            want = ref_port.runfile_text(fused, tags[key])
        else:
            name = key[len("learned_"):]
            f = str(model_files[name])
            if mlp.model_kind(f) == "FusionMLP":
                model = mlp.load_mlp_model(f)
                wd = mlp_oracle.weights_dict(frames, qpp, model)
                n_r = len(model.retrievers)  # src/fusion.py:415 n_retrievers
            else:
                model = lgbm.load_fusion_model(f)
                wd = lgbm_oracle.weights_dict(frames, qpp, model)
                n_r = len(model.retrievers)
            fused = ref_port.learned_fusion_from_weights(frames, wd, n_r)
            want = ref_port.runfile_text(fused, f"learned-{name}")
        ok[key] = _file_rows(path, qids) == want
    return ok


def check_eval(fused_dir: Path, qrels_path: Path, results_json: List[dict]) -> bool:
    """comparison_results.json == the C trec_eval restatement's means, metric by metric.
    Each file's rows straight from the native loader (qfio, the values float() gives),
    documents coded in one sorted table with the qrels' (no per-row Python tuples)."""
    from oracle import _loader as coracle
    from qppfuse.config import config
    from qppfuse.data_utils import load_qrels
    from qppfuse.fastio import read_run_rows
    qrels = load_qrels(qrels_path)
    names = config.evaluation.ir_metrics[:6]
    by_method = {r["method"]: r for r in results_json}
    for res_file in sorted(fused_dir.glob("*.res")):
        print(f"[check_eval] {res_file.name}", file=sys.stderr, flush=True)
        qids, docnos, rq, rd, rr, rsc = read_run_rows(str(res_file))
        # queries in first-appearance order, those with qrels (06: q in qrels)
        _, first = np.unique(rq, return_index=True)
        qorder = np.argsort(first, kind="stable")
        keep = np.array([str(qids[c]) in qrels for c in qorder], dtype=bool)
        qsel = qorder[keep]
        pos = np.full(len(qids), -1, np.int64)
        pos[qsel] = np.arange(len(qsel))
        rows = np.flatnonzero(pos[rq] >= 0)
        qrel_docs = [d for c in qsel for d in qrels[str(qids[c])]]
        table = np.unique(np.concatenate([docnos, np.asarray(qrel_docs, dtype=object)]))
        did = np.searchsorted(table, docnos).astype(np.uint32)
        order = rows[np.argsort(pos[rq[rows]], kind="stable")]
        cnt = np.bincount(pos[rq[order]], minlength=len(qsel))
        roff = np.zeros(len(qsel) + 1, np.int64)
        np.cumsum(cnt, out=roff[1:])
        qo, qd, qr = [0], [], []
        for c in qsel:
            for d, rel in qrels[str(qids[c])].items():
                qd.append(int(np.searchsorted(table, d)))
                qr.append(rel)
            qo.append(len(qd))
        vals = coracle.evaluate(roff, did[rd[order]], rsc[order], np.array(qo, np.int64),
                                np.array(qd, np.uint32), np.array(qr, np.int32), names,
                                text=True)
        got = by_method[res_file.stem]
        for t, name in enumerate(names):
            col = vals[:, t]
            col = col[~np.isnan(col)]
            want = float(col.mean()) if col.size else 0.0
            if abs(got[name] - want) > 1e-12:
                return False
        if got["n_queries"] != len(qsel):
            return False
    return True

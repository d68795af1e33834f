#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container only (the GPU box has no /root/reference):
    python tests/golden/make_golden.py
It imports the reference's own src/fusion.py, src/qpp.py, src/data_utils.py,
src/config.py and src/retrievers/base.py by file path — with a bare `src`
package (src/__init__.py:33 pulls ir_measures, not installed) and a stub `ranx`
module (not installed; only its three names are bound at import) — runs them on
small synthetic inputs, and writes inputs + outputs as JSON / text.  Nothing of
the reference's source is copied: the fixtures are data.  Floats are stored
with float.hex() so the comparison can be bit-exact.

What is pinned here (see DESIGN.md "Parity"):
  weighted_combsum / weighted_combmnz / weighted_rrf (incl. ties, missing
  rankers, qpp_index=-1, unsorted rows), write_runfile bytes, get_qpp_index,
  get_qpp_weight errors, _normalize_qpp, normalize_scores, load_qpp_scores,
  load_runs, and the committed .qpp text columns 7-8 with their query texts.
"""
from __future__ import annotations

import importlib.util
import io
import json
import os
import random
import shutil
import sys
import tempfile
import types
from contextlib import redirect_stdout
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def load_reference():
    tmp = tempfile.mkdtemp(prefix="qppfuse_ref_")
    os.environ["PROJECT_ROOT"] = tmp  # src/config.py:202-203 mkdirs cache_root
    src = types.ModuleType("src")
    src.__path__ = [str(REF / "src")]
    sys.modules["src"] = src
    ranx = types.ModuleType("ranx")
    ranx.Run = ranx.fuse = ranx.Qrels = None
    sys.modules["ranx"] = ranx

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    mods = {}
    mods["config"] = load("src.config", REF / "src/config.py")
    mods["data_utils"] = load("src.data_utils", REF / "src/data_utils.py")
    mods["fusion"] = load("src.fusion", REF / "src/fusion.py")
    mods["qpp"] = load("src.qpp", REF / "src/qpp.py")
    mods["base"] = load("src.retrievers.base", REF / "src/retrievers/base.py")
    return mods


def hx(x: float) -> str:
    return float(x).hex()


def make_case(rng, n_q, rankers, k_range, pool, p_skip=0.0, ties=False, unsorted=False,
              neg=False, rank_shift=False, normed=False):
    """Synthetic .norm.res-like runs: {ranker: rows}; rows = [qid, docno, rank, score]."""
    runs = {}
    qids = [f"test{i}" for i in rng.sample(range(1000), n_q)]
    for r in rankers:
        rows = []
        for qid in qids:
            if rng.random() < p_skip:
                continue
            k = rng.randint(*k_range)
            docs = rng.sample(pool, k)
            if ties:
                vals = sorted((rng.randint(0, 4) / 4 for _ in range(k)), reverse=True)
            else:
                vals = sorted((rng.randint(0, 10**6) / 1e6 for _ in range(k)), reverse=True)
                vals = [float(f"{v:.6f}") for v in vals]
            if neg:
                vals = [v - 0.5 for v in vals]
            if normed and len(vals) > 1 and vals[0] > vals[-1]:
                # a .norm.res list: per-query min-max, written "%.6f"
                lo, hi = vals[-1], vals[0]
                vals = [float(f"{(v - lo) / (hi - lo):.6f}") for v in vals]
            items = [[qid, d, i + 1 + (3 if rank_shift else 0), v]
                     for i, (d, v) in enumerate(zip(docs, vals))]
            if unsorted:
                rng.shuffle(items)
            rows.extend(items)
        runs[r] = rows
    return qids, runs


def to_frames(runs):
    import pandas as pd
    out = {}
    for r, rows in runs.items():
        df = pd.DataFrame(rows, columns=["qid", "docno", "rank", "score"])
        df.insert(1, "iter", "Q0")
        df["runid"] = r
        df["qid"] = df["qid"].astype(str)
        out[r] = df
    return out


def make_qpp(rng, qids, rankers, const=None, missing=None):
    data = {}
    for q in qids:
        data[q] = {}
        for r in rankers:
            if missing and (q, r) == missing:
                continue
            if const is not None:
                data[q][r] = [const] * 13
            else:
                data[q][r] = [float(f"{rng.random():.6f}") for _ in range(13)]
    return data


def enc_fused(fused):
    return {q: [[d, hx(s)] for d, s in lst] for q, lst in fused.items()}


def main():
    mods = load_reference()
    fu, qp, du, base = mods["fusion"], mods["qpp"], mods["data_utils"], mods["base"]
    rng = random.Random(20251212)
    pool = [f"doc{i}" for i in range(60)]
    rankers = ["BGE", "BM25", "Splade"]

    cases = []
    specs = [
        ("basic", dict(n_q=6, rankers=rankers, k_range=(5, 12), pool=pool), dict(), 5),
        ("fusion_mode", dict(n_q=5, rankers=rankers, k_range=(4, 10), pool=pool), dict(), -1),
        ("ties", dict(n_q=5, rankers=rankers, k_range=(6, 14), pool=pool[:20], ties=True),
         dict(), 3),
        ("missing_rows", dict(n_q=7, rankers=rankers, k_range=(3, 9), pool=pool, p_skip=0.3),
         dict(), 5),
        ("unsorted_rankshift", dict(n_q=4, rankers=rankers, k_range=(5, 9), pool=pool,
                                    unsorted=True, rank_shift=True), dict(), 5),
        ("negative_zero_weight", dict(n_q=4, rankers=rankers, k_range=(5, 9), pool=pool,
                                      neg=True), dict(const=0.0), 5),
        ("unit_weights", dict(n_q=6, rankers=rankers + ["BM25_TCT", "BM25_MonoT5"],
                              k_range=(8, 20), pool=pool, normed=True), dict(const=1.0), 5),
        ("five_rankers", dict(n_q=8, rankers=["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade"],
                              k_range=(15, 40), pool=[f"d{i}" for i in range(120)], normed=True),
         dict(), 5),
    ]
    for name, cspec, qspec, qidx in specs:
        qids, runs = make_case(rng, **cspec)
        qpp = make_qpp(rng, qids, cspec["rankers"], **qspec)
        frames = to_frames(runs)
        case = {"name": name, "rankers": cspec["rankers"], "runs": runs, "qpp": qpp,
                "qpp_index": qidx, "rrf_k": 60, "outputs": {}, "runfiles": {}}
        with redirect_stdout(io.StringIO()):
            outs = {
                "wcombsum": fu.weighted_combsum(frames, qpp, qidx),
                "wcombmnz": fu.weighted_combmnz(frames, qpp, qidx),
                "wrrf": fu.weighted_rrf(frames, qpp, qidx, k=60),
            }
            for m, fused in outs.items():
                case["outputs"][m] = enc_fused(fused)
                with tempfile.NamedTemporaryFile("r", suffix=".res", delete=False) as tf:
                    path = tf.name
                fu.write_runfile(fused, path, f"{m}-tag")
                case["runfiles"][m] = Path(path).read_text()
                os.unlink(path)
        cases.append(case)

    # errors of get_qpp_weight (missing qid / ranker even without rows, bad index)
    qids, runs = make_case(rng, n_q=3, rankers=rankers, k_range=(3, 5), pool=pool)
    frames = to_frames(runs)
    errors = []
    for label, qpp, qidx in [
        ("missing_ranker", make_qpp(rng, qids, rankers, missing=(sorted(qids)[1], "BM25")), 5),
        ("missing_qid", {q: v for q, v in make_qpp(rng, qids, rankers).items()
                         if q != sorted(qids)[2]}, 5),
        ("bad_index", make_qpp(rng, qids, rankers), 13),
    ]:
        try:
            with redirect_stdout(io.StringIO()):
                fu.weighted_combsum(frames, qpp, qidx)
            err = None
        except Exception as exc:  # noqa: BLE001
            err = [type(exc).__name__, str(exc)]
        errors.append({"label": label, "runs": runs, "qpp": qpp, "qpp_index": qidx,
                       "error": err})

    # qid sort key of write_runfile with mixed qids
    mixed = {}
    try:
        with redirect_stdout(io.StringIO()):
            fu.write_runfile({"test3": [("a", 1.0)], "5ae7": [("b", 1.0)]}, os.devnull, "t")
        mixed["error"] = None
    except Exception as exc:  # noqa: BLE001
        mixed["error"] = [type(exc).__name__, str(exc)]

    # get_qpp_index
    names = ["RSD", "rsd", "NQC", "nqc", "Sigma(%)", "sigma_max", "QPP-PRP", "WIG", "SCNQC",
             "QV-NQC", "DM", "NQA-QPP", "BERTQPP", "SMV", "UEF", "fusion", "FUSION", "bogus"]
    idx = {}
    for n in names:
        try:
            idx[n] = fu.get_qpp_index(n)
        except Exception as exc:  # noqa: BLE001
            idx[n] = [type(exc).__name__]

    # _normalize_qpp (minmax) on raw predictor rows, incl. a constant column
    raw = {}
    for i in range(25):
        row = [rng.uniform(-3, 5) for _ in range(13)]
        row[12] = 0.25  # constant column -> scale 1.0 -> zeros
        raw[str(i) if i % 2 else f"q{i}"] = row
    norm = qp._normalize_qpp(raw, "minmax")
    normq = {"raw": {q: [hx(v) for v in r] for q, r in raw.items()},
             "norm": {q: [hx(float(v)) for v in r] for q, r in norm.items()}}

    # normalize_scores
    lists = [[(f"d{i}", rng.uniform(-20, 40), i + 1) for i in range(n)] for n in (1, 2, 7, 30)]
    lists.append([("a", 3.5, 1), ("b", 3.5, 2), ("c", 3.5, 3)])
    lists.append([])
    ns = [{"in": [[d, hx(s), r] for d, s, r in L],
           "out": [[d, hx(s), r] for d, s, r in base.BaseRetriever.normalize_scores(L)]}
          for L in lists]

    # loaders on files written here
    tmp = Path(tempfile.mkdtemp(prefix="qppfuse_files_"))
    (tmp / "runs").mkdir()
    (tmp / "qpp").mkdir()
    for r, rows in cases[0]["runs"].items():
        with open(tmp / "runs" / f"{r}.norm.res", "w") as fh:
            for qid, d, rk, s in rows:
                fh.write(f"{qid} Q0 {d} {rk} {s:.6f} {r}\n")
        with open(tmp / "qpp" / f"{r}.res.mmnorm.qpp", "w") as fh:
            for qid, vals in cases[0]["qpp"].items():
                fh.write(qid + "\t" + "\t".join(f"{v:.6f}" for v in vals[r]) + "\n")
    files = {"runs": {f"{r}.norm.res": (tmp / "runs" / f"{r}.norm.res").read_text()
                      for r in cases[0]["runs"]},
             "qpp": {f"{r}.res.mmnorm.qpp": (tmp / "qpp" / f"{r}.res.mmnorm.qpp").read_text()
                     for r in cases[0]["runs"]}}
    loaded_qpp = du.load_qpp_scores(tmp / "qpp")
    loaded_runs = fu.load_runs(str(tmp / "runs"))
    files["load_qpp_scores"] = {q: {r: [hx(v) for v in vals] for r, vals in d.items()}
                                for q, d in loaded_qpp.items()}
    files["load_runs"] = {r: {"qid": df["qid"].tolist(), "docno": df["docno"].tolist(),
                              "rank": [int(x) for x in df["rank"]],
                              "score": [hx(x) for x in df["score"]]}
                          for r, df in loaded_runs.items()}
    with redirect_stdout(io.StringIO()):
        fused = fu.run_fusion("wcombsum", str(tmp / "runs"), str(tmp / "qpp"), "RSD", None,
                              str(tmp / "wcs.res"), 60)
    files["run_fusion_wcombsum_rsd"] = (tmp / "wcs.res").read_text()
    shutil.rmtree(tmp)

    golden = {"cases": cases, "errors": errors, "mixed_qids": mixed, "qpp_index": idx,
              "normalize_qpp": normq, "normalize_scores": ns, "files": files}
    (OUT / "reference_fusion.json").write_text(json.dumps(golden, indent=1, sort_keys=True))

    # committed .qpp text columns 7-8 (MaxIDF / avgidf proxies) + their query texts
    for ds, qdir in [("scifact", "BEIR-scifact"), ("nq", "BEIR-nq")]:
        texts = {}
        with open(REF / "data" / ds / qdir / "queries.jsonl") as fh:
            for line in fh:
                q = json.loads(line)
                texts[q["_id"]] = q["text"]
        cols = {}
        for line in open(REF / "data" / ds / "qpp" / "BGE.res.mmnorm.qpp"):
            f = line.rstrip("\n").split("\t")
            cols[f[0]] = [f[8], f[9], f[12], f[13]]  # cols 7, 8, 11, 12 as written
        fixture = {"qids": list(cols.keys()), "text": [texts.get(q, q) for q in cols],
                   "col7": [cols[q][0] for q in cols], "col8": [cols[q][1] for q in cols],
                   "col11": [cols[q][2] for q in cols], "col12": [cols[q][3] for q in cols]}
        (OUT / f"qpp_textcols_{ds}.json").write_text(json.dumps(fixture))
    print("golden fixtures written to", OUT)
    round2(mods)


def beir_qids():
    """Unique qids of the three BEIR test qrels, in file order (src/data_utils.py:175-197)."""
    out = {}
    for ds in ("hotpotqa", "nq", "scifact"):
        seen = {}
        with open(REF / "data" / ds / f"BEIR-{ds}" / "qrels" / "test.tsv") as fh:
            next(fh)
            for line in fh:
                f = line.strip().split("\t")
                if len(f) >= 3:
                    seen.setdefault(f[0], None)
        out[ds] = list(seen)
    return out


def round2(mods):
    """Fixtures added in round 2 (separate file, so the round-1 vectors stay byte-stable):
      dup_cases   docnos repeated inside one list: the weighted loops (every row
                  counts, src/fusion.py:273-277,321-324,372-374), write_runfile bytes,
                  and _df_runs_to_ranx's {qid: {docno: score}} (last row wins at the
                  first row's position, src/fusion.py:459-464) through a recording
                  stand-in for ranx.Run (ranx is not installed; Run only stores the dict)
      config      the reference's outputs with its config singleton set to
                  rrf_k=20, default_index=7, default_method="WIG" (what a user's
                  edited defaults.yaml gives): weighted_* and run_fusion with no
                  explicit qpp_index / k / qpp_model
      qids        write_runfile's qid order for the namespaced ("<corpus>:<qid>")
                  real BEIR test qids of HotpotQA + NQ + SciFact, and the TypeError
                  of the bare mixed qids (src/fusion.py:487)
    """
    import gzip
    fu, cfgmod = mods["fusion"], mods["config"]
    rng = random.Random(20251213)
    pool = [f"doc{i}" for i in range(40)]
    rankers = ["BGE", "BM25", "Splade"]

    class RecRun(dict):
        def __init__(self, d, name=None):
            super().__init__(d)
            self.name = name
    fu.Run = RecRun

    def dup_runs(n_q, k_range, p_dup, unsorted=False, rank_shift=False):
        qids, runs = make_case(rng, n_q=n_q, rankers=rankers, k_range=k_range, pool=pool,
                               normed=True, unsorted=unsorted, rank_shift=rank_shift)
        for r in rankers:
            rows = runs[r]
            extra = []
            used = {(row[0], row[2]) for row in rows}
            for row in rows:
                if rng.random() < p_dup:
                    for _ in range(rng.choice((1, 1, 2))):
                        # a rank no other row of the list holds: W-RRF's
                        # sort_values("rank") is numpy's unstable quicksort, whose
                        # order among equal ranks is not reproducible
                        rk = rng.randint(1, 40)
                        while (row[0], rk) in used:
                            rk = rng.randint(1, 40)
                        used.add((row[0], rk))
                        extra.append([row[0], row[1], rk, float(f"{rng.random():.6f}")])
            for e in extra:  # inserted at random places of the same query's rows
                idx = [i for i, x in enumerate(rows) if x[0] == e[0]]
                rows.insert(rng.choice(idx) + rng.randint(0, 1), e)
        return qids, runs

    dup_cases = []
    for name, spec in [("dup_basic", dict(n_q=5, k_range=(5, 12), p_dup=0.25)),
                       ("dup_unsorted", dict(n_q=4, k_range=(5, 10), p_dup=0.3, unsorted=True,
                                             rank_shift=True)),
                       ("dup_heavy", dict(n_q=3, k_range=(8, 15), p_dup=0.6))]:
        qids, runs = dup_runs(**spec)
        qpp = make_qpp(rng, qids, rankers)
        frames = to_frames(runs)
        case = {"name": name, "rankers": rankers, "runs": runs, "qpp": qpp, "qpp_index": 5,
                "rrf_k": 60, "outputs": {}, "runfiles": {}}
        with redirect_stdout(io.StringIO()):
            outs = {"wcombsum": fu.weighted_combsum(frames, qpp, 5),
                    "wcombmnz": fu.weighted_combmnz(frames, qpp, 5),
                    "wrrf": fu.weighted_rrf(frames, qpp, 5, k=60)}
            for m, fused in outs.items():
                case["outputs"][m] = enc_fused(fused)
                with tempfile.NamedTemporaryFile("r", suffix=".res", delete=False) as tf:
                    path = tf.name
                fu.write_runfile(fused, path, f"{m}-tag")
                case["runfiles"][m] = Path(path).read_text()
                os.unlink(path)
        rx = fu._df_runs_to_ranx(frames)
        case["ranx_input"] = {r: {q: [[d, hx(v)] for d, v in dq.items()] for q, dq in run.items()}
                              for r, run in rx.items()}
        dup_cases.append(case)

    # config: the singleton's values as an edited defaults.yaml would set them
    c = cfgmod.config._data
    saved = (c.fusion.rrf_k, c.qpp.default_index, c.qpp.default_method)
    c.fusion.rrf_k, c.qpp.default_index, c.qpp.default_method = 20, 7, "WIG"
    qids, runs = make_case(rng, n_q=5, rankers=rankers, k_range=(6, 12), pool=pool, normed=True)
    qpp = make_qpp(rng, qids, rankers)
    frames = to_frames(runs)
    conf = {"yaml": {"fusion": {"rrf_k": 20}, "qpp": {"default_index": 7, "default_method": "WIG"}},
            "runs": runs, "rankers": rankers, "qpp": qpp, "outputs": {}}
    tmp = Path(tempfile.mkdtemp(prefix="qppfuse_cfg_"))
    (tmp / "runs").mkdir()
    (tmp / "qpp").mkdir()
    for r, rows in runs.items():
        with open(tmp / "runs" / f"{r}.norm.res", "w") as fh:
            for qid, d, rk, sc in rows:
                fh.write(f"{qid} Q0 {d} {rk} {sc:.6f} {r}\n")
        with open(tmp / "qpp" / f"{r}.res.mmnorm.qpp", "w") as fh:
            for qid, vals in qpp.items():
                fh.write(qid + "\t" + "\t".join(f"{v:.6f}" for v in vals[r]) + "\n")
    with redirect_stdout(io.StringIO()):
        conf["outputs"]["wcombsum"] = enc_fused(fu.weighted_combsum(frames, qpp))
        conf["outputs"]["wrrf"] = enc_fused(fu.weighted_rrf(frames, qpp))
        fu.run_fusion("wrrf", str(tmp / "runs"), str(tmp / "qpp"), None, None,
                      str(tmp / "wrrf.res"), None)
    conf["run_fusion_wrrf"] = (tmp / "wrrf.res").read_text()
    conf["qpp_files"] = {f.name: f.read_text() for f in sorted((tmp / "qpp").iterdir())}
    shutil.rmtree(tmp)
    c.fusion.rrf_k, c.qpp.default_index, c.qpp.default_method = saved

    # namespaced multi-corpus qids
    bq = beir_qids()
    (OUT / "beir_qids.json.gz").write_bytes(gzip.compress(json.dumps(bq).encode(), mtime=0))
    ns = [f"{ds}:{q}" for ds in ("nq", "scifact", "hotpotqa") for q in bq[ds]]
    with tempfile.NamedTemporaryFile("r", suffix=".res", delete=False) as tf:
        path = tf.name
    with redirect_stdout(io.StringIO()):
        fu.write_runfile({q: [("d", 1.0)] for q in ns}, path, "t")
    order = [line.split(" ", 1)[0] for line in Path(path).read_text().splitlines()]
    os.unlink(path)
    qids_fx = {"namespaced_input": "nq, scifact, hotpotqa blocks in qrels order",
               "namespaced_order": [ns.index(q) for q in order]}
    try:
        with redirect_stdout(io.StringIO()):
            fu.write_runfile({q: [("d", 1.0)] for ds in ("nq", "scifact", "hotpotqa")
                              for q in bq[ds]}, os.devnull, "t")
        qids_fx["bare_error"] = None
    except Exception as exc:  # noqa: BLE001
        qids_fx["bare_error"] = [type(exc).__name__, str(exc)]
    per = {}
    for ds in ("nq", "scifact", "hotpotqa"):
        with tempfile.NamedTemporaryFile("r", suffix=".res", delete=False) as tf:
            path = tf.name
        with redirect_stdout(io.StringIO()):
            fu.write_runfile({q: [("d", 1.0)] for q in bq[ds]}, path, "t")
        got = [line.split(" ", 1)[0] for line in Path(path).read_text().splitlines()]
        os.unlink(path)
        per[ds] = [bq[ds].index(q) for q in got]
    qids_fx["per_corpus_order"] = per
    (OUT / "reference_round2.json").write_text(json.dumps(
        {"dup_cases": dup_cases, "config": conf, "qids": qids_fx}, indent=1, sort_keys=True))
    print("round-2 fixtures written to", OUT)


def round3(mods):
    """Fixtures added in round 3 (reference_round3.json):
      write_run   scripts/02_retrieve.py:65-82 on {qid: RetrieverResult} — the
                  reference's own RetrieverResult and BaseRetriever.normalize_scores
                  (src/retrievers/base.py:14-21,60-73), and the 12-line loop of
                  write_run restated here (02_retrieve.py imports faiss at :34, not
                  installed).  Raw, unrounded scores (BM25-like, dense-like,
                  negative MonoT5-like), ties, a constant list, an empty list, one
                  entry; normalize True and False; the bytes written.
    """
    base = mods["base"]
    rng = random.Random(20251214)

    def restated_write_run(results, output_path, retriever_name, normalize=False):
        os.makedirs(os.path.dirname(output_path), exist_ok=True)
        with open(output_path, "w") as f:
            for qid in sorted(results.keys(),
                              key=lambda x: int(x.replace("test", "")) if x.startswith("test") else x):
                docs = results[qid].results
                if normalize:
                    docs = base.BaseRetriever.normalize_scores(docs)
                for docno, score, rank in docs:
                    f.write(f"{qid} Q0 {docno} {rank} {score:.6f} {retriever_name}\n")

    def lists(kind, n_q):
        out = {}
        for q in range(n_q):
            qid = f"test{rng.randrange(0, 5000)}"
            while qid in out:
                qid = f"test{rng.randrange(0, 5000)}"
            k = rng.choice((1, 2, 7, 25, 60))
            if kind == "bm25":
                sc = sorted((rng.gammavariate(2.0, 6.0) + 5.0 for _ in range(k)), reverse=True)
            elif kind == "dense":
                sc = sorted((0.5 + 0.4 * rng.betavariate(5, 2) for _ in range(k)), reverse=True)
            elif kind == "monot5":
                sc = sorted((-rng.expovariate(0.3) for _ in range(k)), reverse=True)
            else:  # ties and a constant list
                v = [rng.choice((0.25, 0.5, 1.0 / 3.0)) for _ in range(k)]
                sc = sorted(v, reverse=True) if q % 2 else [v[0]] * k
            docs = [(f"doc{rng.randrange(10 ** 6)}", s, i + 1) for i, s in enumerate(sc)]
            out[qid] = docs
        out[f"test{5000 + n_q}"] = []  # a query with no documents
        return out

    cases = []
    for kind, name in (("bm25", "BM25"), ("dense", "BGE"), ("monot5", "BM25_MonoT5"),
                       ("ties", "Splade")):
        raw = lists(kind, 9)
        for normalize in (True, False):
            res = {q: base.RetrieverResult(qid=q, results=list(d), retriever_name=name)
                   for q, d in raw.items()}
            tmp = Path(tempfile.mkdtemp(prefix="qppfuse_wr_"))
            path = tmp / "runs" / "nested" / f"{name}{'.norm' if normalize else ''}.res"
            restated_write_run(res, str(path), name, normalize=normalize)
            cases.append({"kind": kind, "retriever_name": name, "normalize": normalize,
                          "results": {q: [[d, hx(s), r] for d, s, r in docs] for q, docs in raw.items()},
                          "expected": path.read_text()})
            shutil.rmtree(tmp)
    (OUT / "reference_round3.json").write_text(json.dumps({"write_run": cases}, indent=1,
                                                          sort_keys=True))
    print("round-3 fixtures written to", OUT)


if __name__ == "__main__":
    if sys.argv[1:] == ["--round3"]:
        round3(load_reference())
    else:
        main()
        round3(load_reference())

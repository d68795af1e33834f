"""End-to-end drop-in timing (development tool; DESIGN.md "End to end").

C2-shaped run files (3,452 queries x 5 retrievers x top-1000, `.norm.res` text)
are generated once, then the reference's fusion entry points are timed through
this package as scripts/05_fusion.py would call them:
  load_runs (native parse) -> load_qpp_scores -> fuse_many (6 methods: H2D,
  qf_fuse, D2H) -> write_runfile x 6 (native writer).
--qpp: the 03_qpp stage instead — five raw `.res` files (the raw scores as
02_retrieve writes them, "%.6f") through compute_qpp_for_res_file into `.qpp`
files: in one warm process, file after file, and as scripts/03_qpp.py runs it
(a fresh Python whose ProcessPoolExecutor gives every file its own worker).
python tools/e2e.py [--queries Q] [--dir DIR] [--qpp]
"""
import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "qpp-fusion-rag_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = ["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade"]
GENERATOR = os.environ.get("E2E_GENERATOR", "nq")  # bench.py's synthetic runs
GOLDEN = ROOT / "tests" / "golden"
MODEL_FILES = {"per_retriever": GOLDEN / "lgbm" / "nq_fusion_per_retriever.json.gz",
               "multioutput": GOLDEN / "lgbm" / "nq_fusion_multioutput.json.gz",
               "mlp": GOLDEN / "mlp" / "nq_fusion_mlp.json.gz"}
METHODS = ["combsum", "combmnz", "rrf", "wcombsum", "wcombmnz", "wrrf"]


def ascii_table(prefix: bytes, ids: np.ndarray):
    """(offsets, bytes) of prefix + decimal(id) for every id, vectorised."""
    ids = ids.astype(np.int64)
    nd = np.maximum(1, np.floor(np.log10(np.maximum(ids, 1))).astype(np.int64) + 1)
    W = int(nd.max())
    dig = np.zeros((len(ids), W), np.uint8)
    v = ids.copy()
    for k in range(W - 1, -1, -1):
        dig[:, k] = 48 + v % 10
        v //= 10
    lens = nd + len(prefix)
    off = np.zeros(len(ids) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    out = np.empty(int(off[-1]), np.uint8)
    pos = off[:-1]
    for i, ch in enumerate(prefix):
        out[pos + i] = ch
    keep = np.arange(W)[None, :] >= (W - nd)[:, None]
    dst = (pos + len(prefix))[:, None] + (np.arange(W)[None, :] - (W - nd)[:, None])
    out[dst[keep]] = dig[keep]
    return off, out.tobytes()


def generate(d: Path, Q: int, R: int, K: int, cpu: bool = False, raw_files: bool = False):
    from qppfuse import fastio
    if cpu:  # no GPU (loader work in the build container): numpy restatement + C oracle
        sys.path.insert(0, str(ROOT / "tools"))
        from synth_np import synth
        from oracle import _loader as coracle
        off_h, doc_h, raw = synth(0, Q, R, K)
        norm = coracle.minmax_per_query(raw, off_h)
        sc_h = np.round(norm * 1e6) / 1e6
        qmicro = np.random.default_rng(1).integers(0, 10**6, (Q * R, 13))
    else:
        from qppfuse import engine
        import bench
        a = SimpleNamespace(generator=GENERATOR)
        off, docid, raw = bench.gen_runs(a, 0, Q, R, K)
        _, micro = engine.minmax_per_query(raw, off, want_norm=False)
        nt = torch.full((Q,), 4, dtype=torch.int32, device=off.device)
        tf = torch.rand((Q, 2), dtype=torch.float64, device=off.device)
        qraw = engine.qpp_raw(raw, off, R, 100, nt, tf)
        mm = engine.qpp_colminmax(qraw, off, R)
        qmicro = engine.qpp_normalize(qraw, mm, off, R, "minmax", 5)["micro"].cpu().numpy()
        off_h = off.cpu().numpy()
        doc_h = docid.cpu().numpy().view(np.uint32)
        sc_h = micro.cpu().numpy().astype(np.float64) / 1e6
    uniq, inv = np.unique(doc_h, return_inverse=True)
    rs = SimpleNamespace(qids=None, docnos=None)
    rs._strtab = {"qid": ascii_table(b"test", np.arange(Q)), "docno": ascii_table(b"doc", uniq)}
    ud = inv.astype(np.uint32)
    pos = (np.arange(len(doc_h)) - np.repeat(off_h[:-1], np.diff(off_h))).astype(np.uint16)
    for r, name in enumerate(NAMES[:R]):
        qb = off_h[r:-1:R][:Q]
        cnt = np.diff(off_h)[r::R][:Q].astype(np.int32)
        fastio.write_run(str(d / f"{name}.norm.res"), np.arange(Q), qb, cnt, ud, pos, sc_h, rs,
                         name)
        if raw_files:  # the raw run 02_retrieve writes beside it (scripts/02_retrieve.py:80)
            raw_h = raw if cpu else raw.cpu().numpy()
            fastio.write_run(str(d / f"{name}.res"), np.arange(Q), qb, cnt, ud, pos, raw_h, rs,
                             name)
    qd = d / "qpp"
    qd.mkdir(exist_ok=True)
    for r, name in enumerate(NAMES[:R]):
        with open(qd / f"{name}.res.mmnorm.qpp", "w") as fh:
            for q in range(Q):
                m = qmicro[q * R + r]
                fh.write(f"test{q}\t" + "\t".join(f"{v // 10**6}.{v % 10**6:06d}" for v in m) + "\n")
    return int(off_h[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=3452)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--qpp", action="store_true", help="time the 03_qpp stage (see above)")
    ap.add_argument("--replay", action="store_true",
                    help="replay scripts/05_fusion.py run_all_methods + 06_eval_fusion.py on the "
                         "files (tests/driver_replay.py) and check a sample of every written file "
                         "byte for byte, and the evaluation JSON, on the CPU reference path")
    ap.add_argument("--sample", type=int, default=64, help="--replay: queries checked per file")
    ap.add_argument("--load-only", action="store_true",
                    help="CPU only: generate with numpy, time load_runs (QFIO_TIMING=1 for phases)")
    a = ap.parse_args()
    from qppfuse import fusion
    d = Path(a.dir or tempfile.mkdtemp(prefix="qf_e2e_"))
    d.mkdir(parents=True, exist_ok=True)
    if a.load_only:
        if not any(d.glob("*.norm.res")):
            generate(d, a.queries, 5, 1000, cpu=True)
        for _ in range(a.repeat):
            t0 = time.perf_counter()
            runs = fusion.load_runs(str(d))
            print(json.dumps({"load_runs_s": round(time.perf_counter() - t0, 4),
                              "rows": int(sum(len(df) for df in runs.values()))}), flush=True)
            del runs
        return
    if a.qpp:
        return qpp_stage(a, d)
    if a.replay:
        return replay(a, d)
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    E = generate(d, a.queries, 5, 1000)
    gen_s = time.perf_counter() - t0
    size = sum(f.stat().st_size for f in d.glob("*.norm.res"))
    best = None
    for _ in range(a.repeat):
        fusion._PACK_CACHE.clear()
        t = {}
        t0 = time.perf_counter()
        runs = fusion.load_runs(str(d))
        t["load_runs_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        qpp = fusion.load_qpp_scores(str(d / "qpp"))
        t["load_qpp_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        res = fusion.fuse_many(runs, METHODS, qpp, 5)
        torch.cuda.synchronize()
        t["fuse_6_methods_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        for m in METHODS:
            fusion.write_runfile(res[m], str(d / f"fused_{m}.res"), m)
        t["write_6_runfiles_s"] = time.perf_counter() - t0
        t["total_s"] = sum(t.values())
        if best is None or t["total_s"] < best["total_s"]:
            best = t
    out_bytes = sum((d / f"fused_{m}.res").stat().st_size for m in METHODS)
    best = {k: round(v, 4) for k, v in best.items()}
    print(json.dumps({"queries": a.queries, "entries": E, "input_bytes": size,
                      "output_bytes": out_bytes, "generate_s": round(gen_s, 2), **best,
                      "e2e_fused_queries_per_s": round(a.queries * 6 / best["total_s"], 1),
                      "cpu_threads": os.cpu_count()}), flush=True)


def replay(a, d: Path):
    """--replay: the reference's driver sequence file to file, checked (module docstring)."""
    import gzip
    sys.path.insert(0, str(ROOT / "tests"))
    import driver_replay as dr
    torch.cuda.set_device(0)
    runs_dir = d / "runs"
    runs_dir.mkdir(exist_ok=True)
    t0 = time.perf_counter()
    if not any(runs_dir.glob("*.norm.res")):
        generate(runs_dir, a.queries, 5, 1000)
    gen_s = time.perf_counter() - t0
    qpp_dir = runs_dir / "qpp"
    fused_dir = d / "fused"
    fused_dir.mkdir(exist_ok=True)
    qrels = d / "test.tsv"
    qrels.write_bytes(gzip.decompress((GOLDEN / "nq_qrels_test.tsv.gz").read_bytes()))
    size = sum(f.stat().st_size for f in runs_dir.glob("*.norm.res"))
    t0 = time.perf_counter()
    results = dr.run_all_methods(runs_dir, qpp_dir, fused_dir, model_files=MODEL_FILES)
    fuse_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    evals = dr.evaluate_fused_runs(fused_dir, qrels, d)
    eval_s = time.perf_counter() - t0
    rng = np.random.default_rng(5)
    sample = [f"test{q}" for q in sorted(rng.choice(a.queries, min(a.sample, a.queries),
                                                    replace=False))]
    t0 = time.perf_counter()
    ok = dr.check_sample(runs_dir, qpp_dir, results, sample, model_files=MODEL_FILES)
    check_s = time.perf_counter() - t0
    eval_ok = dr.check_eval(fused_dir, qrels, evals)
    out_bytes = sum(p.stat().st_size for p in results.values())
    print(json.dumps({"stage": "05_fusion.run_all_methods + 06_eval_fusion.evaluate_fused_runs",
                      "queries": a.queries, "input_bytes": size, "output_bytes": out_bytes,
                      "files": sorted(p.name for p in results.values()),
                      "generate_s": round(gen_s, 2), "run_all_methods_s": round(fuse_s, 3),
                      "evaluate_fused_runs_s": round(eval_s, 3),
                      "sample_queries": len(sample), "bytes_equal_per_file": ok,
                      "bytes_equal": all(ok.values()), "check_s": round(check_s, 1),
                      "eval_equal_oracle": eval_ok,
                      "ndcg10": {r["method"]: round(r["nDCG@10"], 5) for r in evals},
                      "generator": GENERATOR, "cpu_threads": os.cpu_count()}), flush=True)


POOL = """
import os, sys
sys.path[:0] = [{root!r}, {pkg!r}]
from concurrent.futures import ProcessPoolExecutor, as_completed
from qppfuse import compute_qpp_for_res_file

def _process_qpp_file(job):  # scripts/03_qpp.py:31-36
    compute_qpp_for_res_file(*job)
    return job[0]

if __name__ == "__main__":
    d, out = sys.argv[1:3]
    jobs = [(os.path.join(d, f), os.path.join(out, f.replace(".res", ".res.mmnorm.qpp")), 100,
             "minmax", None) for f in sorted(os.listdir(d))
            if f.endswith(".res") and not f.endswith(".norm.res")]
    with ProcessPoolExecutor(max_workers=min(8, len(jobs))) as ex:
        for fut in as_completed([ex.submit(_process_qpp_file, j) for j in jobs]):
            fut.result()
"""


def qpp_stage(a, d: Path):
    """The 03_qpp stage file to file (see the module docstring)."""
    import subprocess
    from qppfuse.qpp import compute_qpp_for_res_file
    torch.cuda.set_device(0)
    if not any(d.glob("*.res")) or not (d / "BGE.res").exists():
        generate(d, a.queries, 5, 1000, raw_files=True)
    files = sorted(f for f in d.glob("*.res") if not f.name.endswith(".norm.res"))
    size = sum(f.stat().st_size for f in files)
    out = d / "qpp_one"
    out.mkdir(exist_ok=True)
    times = []
    for _ in range(a.repeat + 1):  # the first pass warms the process (HIP context, caches)
        t0 = time.perf_counter()
        for f in files:
            compute_qpp_for_res_file(str(f), str(out / f.name.replace(".res", ".res.mmnorm.qpp")))
        times.append(time.perf_counter() - t0)
    pool = d / "qpp_pool"
    pool.mkdir(exist_ok=True)
    script = d / "qpp03_pool.py"
    script.write_text(POOL.format(root=str(ROOT), pkg=str(ROOT / "qpp-fusion-rag_amd")))
    t0 = time.perf_counter()
    subprocess.run([sys.executable, str(script), str(d), str(pool)], check=True,
                   stdout=subprocess.DEVNULL)
    pool_s = time.perf_counter() - t0
    same = all((pool / f.name.replace(".res", ".res.mmnorm.qpp")).read_bytes() ==
               (out / f.name.replace(".res", ".res.mmnorm.qpp")).read_bytes() for f in files)
    print(json.dumps({"stage": "03_qpp", "files": len(files), "queries": a.queries,
                      "input_bytes": size, "first_pass_s": round(times[0], 4),
                      "warm_process_s": round(min(times[1:]), 4),
                      "process_pool_wall_s": round(pool_s, 3),
                      "pool_qpp_bytes_equal_single_process": same,
                      "cpu_threads": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()

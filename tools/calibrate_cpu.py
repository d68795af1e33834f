"""Calibrate bench.py's CPU baseline (oracle/ref_port.py, timed on the GPU box) against
the reference itself, on ONE host: this build container, which has /root/reference.

Imports the reference's src/fusion.py the way tests/golden/make_golden.py does (bare
`src` package, stub `ranx`), builds a 200-query C2-shaped sample (5 retrievers x
top-1000, tools/synth_np.py: the bench's synthetic generator restated), and times,
single-threaded, the reference's weighted_combsum / weighted_rrf and ref_port's
restatement of the same functions on the same frames.  Writes
profiles/r03_cpu_calibration.json: microseconds per row of each, and the ratio
reference / port that bench.py applies to its live port timing.
Usage (build container only): python tools/calibrate_cpu.py [n_queries]
"""
import io
import json
import os
import platform
import sys
import time
from contextlib import redirect_stdout
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tools"), str(ROOT / "tests" / "golden")]
os.environ["OMP_NUM_THREADS"] = "1"
import numpy as np
import pandas as pd

from make_golden import load_reference
from oracle import _loader as coracle
from oracle import ref_port
from synth_np import synth

NAMES = ["BGE", "BM25", "BM25_MonoT5", "BM25_TCT", "Splade"]


def main():
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    R, K = 5, 1000
    off, docid, raw = synth(0, nq, R, K)
    norm = coracle.minmax_per_query(raw, off)
    micro = np.array([int(f"{v:.6f}".replace(".", "")) for v in norm], np.int64)
    qids = [f"test{q}" for q in range(nq)]
    frames = {}
    for r, name in enumerate(NAMES):
        rows_q, rows_d, rows_r, rows_s = [], [], [], []
        for q in range(nq):
            a, b = off[q * R + r], off[q * R + r + 1]
            rows_q += [qids[q]] * (b - a)
            rows_d += [f"doc{d}" for d in docid[a:b]]
            rows_r += list(range(1, b - a + 1))
            rows_s += (micro[a:b] / 1e6).tolist()
        frames[name] = pd.DataFrame({"qid": rows_q, "iter": "Q0", "docno": rows_d,
                                     "rank": rows_r, "score": rows_s, "runid": name})
    rows = sum(len(df) for df in frames.values())
    rng = np.random.default_rng(3)
    qpp = {q: {n: rng.random(13).tolist() for n in NAMES} for q in qids}
    fu = load_reference()["fusion"]
    out = {"sample": f"{nq} queries x {R} retrievers x top-{K} ({rows} rows), "
                     "tools/synth_np.py (bench.py's synthetic generator restated)",
           "host": f"{platform.processor() or platform.machine()}, {os.cpu_count()} CPUs "
                   "(build container), 1 thread",
           "reference_us_per_row": {}, "port_us_per_row": {}, "ratio_reference_over_port": {}}
    for m, ref_fn in (("wcombsum", lambda: fu.weighted_combsum(frames, qpp, 5)),
                      ("wrrf", lambda: fu.weighted_rrf(frames, qpp, 5, k=60))):
        with redirect_stdout(io.StringIO()):
            t0 = time.perf_counter()
            want = ref_fn()
            t_ref = time.perf_counter() - t0
        t0 = time.perf_counter()
        got = ref_port.fuse(frames, m, qpp, 5, 60)
        t_port = time.perf_counter() - t0
        assert {q: list(v) for q, v in got.items()} == {q: list(v) for q, v in want.items()}, m
        out["reference_us_per_row"][m] = round(t_ref / rows * 1e6, 3)
        out["port_us_per_row"][m] = round(t_port / rows * 1e6, 3)
        out["ratio_reference_over_port"][m] = round(t_ref / t_port, 4)
        print(m, out["reference_us_per_row"][m], out["port_us_per_row"][m],
              out["ratio_reference_over_port"][m], flush=True)
    r = out["ratio_reference_over_port"]
    out["ratio"] = round(float(np.mean(list(r.values()))), 4)
    out["note"] = ("bench.py times ref_port on the GPU box's cores; multiplying its time by "
                   "`ratio` (dividing its rate) estimates the reference itself there. The "
                   "outputs of the two were checked equal on this sample.")
    (ROOT / "profiles" / "r03_cpu_calibration.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()

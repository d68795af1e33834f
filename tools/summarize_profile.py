"""Turn a tools/profile.sh output directory into committed summaries under profiles/.

python tools/summarize_profile.py gpurun_out/prof r01
 -> profiles/r01_kernel_stats.csv  (rocprofv3 --kernel-trace --stats, verbatim)
    profiles/r01_pmc.json          (per-kernel mean FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU per launch:
                                    write bytes = WRITE_SIZE x 1024, read bytes = FETCH_SIZE x 1024
                                    x 2 — the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE
                                    tallies 128-B requests at 64 B), checked here on the min-max
                                    kernel, whose reads are a known byte count: every raw f64 score
                                    of the C2 run set once + the list offsets)
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

src, tag = Path(sys.argv[1]), sys.argv[2]
out = Path(__file__).resolve().parents[1] / "profiles"
out.mkdir(exist_ok=True)
shutil.copy(src / "trace" / "run_kernel_stats.csv", out / f"{tag}_kernel_stats.csv")
pmc = collections.defaultdict(dict)
for name in ("fetch", "write", "valu"):
    f = src / name / "run_counter_collection.csv"
    if not f.exists():
        continue
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(list)
    for r in rows:
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in agg.items():
        pmc[k][c] = {"mean_kb_per_launch": sum(v) / len(v), "launches": len(v)}
stats = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(src / "trace" / "run_kernel_stats.csv"))}
FETCH_X = 2.0  # gfx950: FETCH_SIZE reports half the bytes of wide coalesced reads
summary = {}
for k, d in pmc.items():
    f = d.get("FETCH_SIZE", {}).get("mean_kb_per_launch")
    w = d.get("WRITE_SIZE", {}).get("mean_kb_per_launch")
    v = d.get("SQ_INSTS_VALU", {}).get("mean_kb_per_launch")  # a count, not KB
    summary[k] = {"fetch_bytes": None if f is None else f * 1024 * FETCH_X,
                  "fetch_size_raw_bytes": None if f is None else f * 1024,
                  "write_bytes": None if w is None else w * 1024,
                  "hbm_bytes": None if f is None or w is None else (f * FETCH_X + w) * 1024,
                  "insts_valu": v,
                  "avg_ns": stats.get(k)}
# qf_fuse = its join kernel + the sort kernels (every launch of one qf_fuse call)
parts = [k for k in summary if any(s in k for s in ("join_kernel", "fuse_kernel", "fuse_large_kernel", "bsort_kernel", "bsort_fast_kernel", "bucket_sort_kernel", "join_sort_kernel", "join_learned_kernel", "join_sort_all_kernel", "join_sort_xl_kernel"))]
if parts:
    tot = lambda f: (None if any(summary[k][f] is None for k in parts)
                     else sum(summary[k][f] for k in parts))
    summary["qf_fuse (sum of its kernels)"] = {
        "kernels": parts, "fetch_bytes": tot("fetch_bytes"), "write_bytes": tot("write_bytes"),
        "hbm_bytes": tot("hbm_bytes"), "insts_valu": tot("insts_valu"),
        "avg_ns": None if any(summary[k]["avg_ns"] is None for k in parts)
        else sum(summary[k]["avg_ns"] for k in parts)}
# the correction checked on a known byte count: the min-max kernel reads every raw f64
# score of the bench's C2 run set once (3,452 x 5 x 1,000) plus the list offsets (the
# fused min-max + QPP column kernel also the 13 raw predictors of every list)
mm = [k for k in summary if "minmax_per_query_kernel" in k or "minmax_colminmax_kernel" in k]
if mm and summary[mm[0]]["fetch_size_raw_bytes"]:
    known = 3452 * 5 * 1000 * 8 + (3452 * 5 + 1) * 8
    if "colminmax" in mm[0]:
        known += 3452 * 5 * 13 * 8
    summary["fetch_calibration"] = {
        "kernel": mm[0], "known_read_bytes": known,
        "fetch_size_raw_bytes": summary[mm[0]]["fetch_size_raw_bytes"],
        "raw_over_known": summary[mm[0]]["fetch_size_raw_bytes"] / known, "factor_applied": FETCH_X}
(out / f"{tag}_pmc.json").write_text(json.dumps(summary, indent=1))
print(json.dumps(summary, indent=1))

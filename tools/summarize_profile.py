"""Turn a tools/profile.sh output directory into committed summaries under profiles/.

python tools/summarize_profile.py gpurun_out/prof r01
 -> profiles/r01_kernel_stats.csv  (rocprofv3 --kernel-trace --stats, verbatim)
    profiles/r01_pmc.json          (per-kernel mean FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU per launch,
                                    bytes = counter x 1024; no gfx950 x2 correction is
                                    applied: calibrated on this pattern)
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
summary = {}
for k, d in pmc.items():
    f = d.get("FETCH_SIZE", {}).get("mean_kb_per_launch")
    w = d.get("WRITE_SIZE", {}).get("mean_kb_per_launch")
    v = d.get("SQ_INSTS_VALU", {}).get("mean_kb_per_launch")  # a count, not KB
    summary[k] = {"fetch_bytes": None if f is None else f * 1024,
                  "write_bytes": None if w is None else w * 1024,
                  "hbm_bytes": None if f is None or w is None else (f + w) * 1024,
                  "insts_valu": v,
                  "avg_ns": stats.get(k)}
# qf_fuse = its join kernel + the sort kernels (every launch of one qf_fuse call)
parts = [k for k in summary if any(s in k for s in ("join_kernel", "fuse_kernel", "fuse_large_kernel", "bucket_sort_kernel", "join_sort_kernel"))]
if parts:
    tot = lambda f: (None if any(summary[k][f] is None for k in parts)
                     else sum(summary[k][f] for k in parts))
    summary["qf_fuse (sum of its kernels)"] = {
        "kernels": parts, "fetch_bytes": tot("fetch_bytes"), "write_bytes": tot("write_bytes"),
        "hbm_bytes": tot("hbm_bytes"), "insts_valu": tot("insts_valu"),
        "avg_ns": None if any(summary[k]["avg_ns"] is None for k in parts)
        else sum(summary[k]["avg_ns"] for k in parts)}
(out / f"{tag}_pmc.json").write_text(json.dumps(summary, indent=1))
print(json.dumps(summary, indent=1))

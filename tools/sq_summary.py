"""Per-kernel mean SQ counters from tools/sqpmc.sh output (development tool)."""
import collections, csv, sys
from pathlib import Path
d = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(d.glob("p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    short = k.split("(")[0][-60:]
    vals = {c: sum(v) / len(v) for c, v in cs.items()}
    print(short)
    print("   " + "  ".join(f"{c[3:]}={v:.3g}" for c, v in sorted(vals.items())))

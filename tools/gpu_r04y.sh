#!/bin/bash
# Round-4 pass W: C5 and C1 kernels — VALU wave-instructions per launch (SQ_INSTS_VALU,
# SQ_WAVES) beside their kernel trace, to place the one-wave sort against the issue roof
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04y
mkdir -p $O
ARGS="--workload c5 --steps 10 --warmup 2 --cpu-sample 0 --native-sample 0 --check 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $ARGS > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/valu -o run -- python3 bench.py $ARGS > $O/valu.log 2>&1 || { tail -20 $O/valu.log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
O = "gpurun_out/r04y"
st = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(glob.glob(O + "/trace/**/run_kernel_stats.csv", recursive=True)[0]))}
agg = collections.defaultdict(list)
for r in csv.DictReader(open(glob.glob(O + "/valu/**/run_counter_collection.csv", recursive=True)[0])):
    agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    if c == "SQ_INSTS_VALU" and ("qf::" in k):
        valu = sum(v) / len(v)
        ns = st.get(k)
        roof_us = valu / (1024 * 0.52) / 1000
        print(f"{k[:70]:70s} valu/launch {valu:.3e}  issue-roof {roof_us:.1f} us  measured {ns/1000 if ns else float('nan'):.1f} us")
PY

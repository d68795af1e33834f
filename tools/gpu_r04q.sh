#!/bin/bash
# Round-4 pass Q: C1's kernels (rocprofv3 kernel trace + stats of the C1 bench line)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c1 -o run -- python3 bench.py --workload c1 --steps 20 --warmup 5 --cpu-sample 0 --native-sample 0 --check 0 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
f=$(find $O/c1 -name "*kernel_stats.csv" | head -1)
cp $f $O/c1_kernel_stats.csv
cut -d, -f1-8 $O/c1_kernel_stats.csv | head -20

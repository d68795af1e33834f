#!/bin/bash
# per-kernel averages of tools/microbench.py under rocprofv3 (kernel trace + stats)
OUT=${1:-gpurun_out/kstats}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/microbench.py > $OUT/micro.log 2>&1

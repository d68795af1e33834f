#!/bin/bash
# Round-4 pass ZA: the one-wave bucket sort at seven waves per SIMD (72 VGPRs, spills) against six
set -e
O=gpurun_out/r04za
mkdir -p $O
for i in 1 2 3; do
  for L in tools/ab/lib_head.so tools/ab/lib_w7.so; do
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
    echo "$i $(basename $L) c1 $(python3 -c "import json; d=json.load(open('$O/c1.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done

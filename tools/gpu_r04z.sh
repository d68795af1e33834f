#!/bin/bash
# Round-4 pass Z: C1's one-wave join with a 512- / 2,048-slot hash table against 1,024
set -e
O=gpurun_out/r04z
mkdir -p $O
for i in 1 2 3; do
  for L in tools/ab/lib_head.so tools/ab/lib_tb9.so tools/ab/lib_tb11.so; do
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
    echo "$i $(basename $L) c1 $(python3 -c "import json; d=json.load(open('$O/c1.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done

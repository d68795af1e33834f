#!/bin/bash
# Round-4 pass T: C1 with a one-wave join (JoinCfg<64, 5, 10>) against the two-wave one
set -e
O=gpurun_out/r04t
mkdir -p $O
for i in 1 2 3; do
  for L in tools/ab/lib_head.so tools/ab/lib_join64.so; do
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
    echo "$i $(basename $L) $(python3 -c "import json; d=json.load(open('$O/c1.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done

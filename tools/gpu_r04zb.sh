#!/bin/bash
# Round-4 pass ZB: the min-max kernels capped at 64 VGPRs (eight waves per SIMD) against
# HEAD — C1 and C2 lines and the C2-shaped per-list min-max
set -e
O=gpurun_out/r04zb
mkdir -p $O
for i in 1 2 3; do
  for L in tools/ab/lib_head.so tools/ab/lib_mm8.so; do
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
    echo "$i $(basename $L) c1 $(python3 -c "import json; d=json.load(open('$O/c1.json')); print(d['ms_per_step'], d['parity_vs_oracle']['bit_exact'])") c2 $(python3 -c "import json; d=json.load(open('$O/c2.json')); print(d['ms_per_step'], d['parity_vs_oracle']['bit_exact'])") $(QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('minmax', d['minmax'])")"
  done
done

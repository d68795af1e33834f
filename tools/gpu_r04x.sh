#!/bin/bash
# Round-4 pass X: a one-wave bucket sort for unions <= 384 (C1; the LSD sort inline as
# its fallback) — the fusion GPU tests, then C1 lines against HEAD's build
set -e
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_boundary.py tests/test_gpu_learned.py tests/test_gpu_eval.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for L in tools/ab/lib_head.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so; do
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
    echo "$i $(basename $L) c1 $(python3 -c "import json; d=json.load(open('$O/c1.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done

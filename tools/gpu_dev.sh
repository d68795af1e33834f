#!/bin/bash
# Development pass on the GPU box: fused-path parity, then per-kernel A/B of the
# working library against libqppfuse_base.so (the last commit), then the C5 step.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_learned.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dev_tests.log 2>&1 || { tail -30 gpurun_out/dev_tests.log; exit 1; }
tail -2 gpurun_out/dev_tests.log
REPS=${REPS:-3} bash tools/ab_kernels.sh qpp-fusion-rag_amd/qppfuse/libqppfuse.so qpp-fusion-rag_amd/qppfuse/libqppfuse_base.so
if [ -n "$C5" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o run -- python3 bench.py --workload c5 --steps 20 --warmup 3 --cpu-sample 0 --native-sample 0 --check 0 > gpurun_out/c5prof.log 2>&1
  python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/c5prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('%-70s %8.1f us x%s' % (r['Name'][:70], float(r['AverageNs'])/1e3, r['Calls']))
PY
  tail -1 gpurun_out/c5prof.log | cut -c1-200
fi

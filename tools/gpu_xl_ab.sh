#!/bin/bash
# A/B of the workspace path: tools/xlbench.py on the working library vs
# libqppfuse_base.so (the last commit), alternating; then the phase stamps.
set -e
mkdir -p gpurun_out/xlab
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py -x -q -k "workspace or wide or capacity or adversarial or more_than" --timeout 200 --timeout-method thread > gpurun_out/xlab/tests.log 2>&1 || { tail -30 gpurun_out/xlab/tests.log; exit 1; }
tail -1 gpurun_out/xlab/tests.log
for i in 1 2; do
  for L in libqppfuse libqppfuse_base; do
    QF_LIB=qpp-fusion-rag_amd/qppfuse/$L.so timeout -k 10 300 python -u tools/xlbench.py ${SHAPE:-500 16 4000} > gpurun_out/xlab/b.log 2>&1 || { tail -20 gpurun_out/xlab/b.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/xlab/b.log').read().strip().splitlines()[-1]); print('$L', {k: v for k, v in d.items() if k.endswith('_ms') or k == 'bit_exact'})"
  done
done
timeout -k 10 300 python -u tools/xlstamps.py ${SHAPE:-500 16 4000} > gpurun_out/xlab/stamps.log 2>&1 && tail -16 gpurun_out/xlab/stamps.log

#!/bin/bash
# Workspace path (queries above 10,240 entries) on the GPU box: parity tests, then
# tools/xlbench.py timings of the working library against libqppfuse_base.so.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/xl
timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/xl/tests.log 2>&1 || { tail -40 gpurun_out/xl/tests.log; exit 1; }
tail -2 gpurun_out/xl/tests.log
for L in qpp-fusion-rag_amd/qppfuse/libqppfuse.so qpp-fusion-rag_amd/qppfuse/libqppfuse_base.so; do
  for shape in "500 16 4000" "3452 16 1000"; do
    QF_LIB=$L timeout -k 10 300 python -u tools/xlbench.py $shape > gpurun_out/xl/bench.log 2>&1 || { tail -20 gpurun_out/xl/bench.log; exit 1; }
    echo "$(basename $L) $(tail -1 gpurun_out/xl/bench.log)"
  done
done

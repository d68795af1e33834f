#!/bin/bash
# Development cycle on the GPU box: fused-path parity, A/B timing, phase stamps.
set -o pipefail
mkdir -p gpurun_out/dev
QF_JS_BLOCK=12 timeout -k 10 120 python tools/jsdebug.py 64 > gpurun_out/dev/jsdbg.log 2>&1 || exit 1
QF_JS_BLOCK=12 timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dev/tests.log 2>&1 || exit 1
tools/ab_js.sh ${JS_BLOCK:-12} 11 13 || exit 1
if [ -f qpp-fusion-rag_amd/qppfuse/libqppfuse_stamps.so ]; then
  QF_JS_BLOCK=${JS_BLOCK:-12} timeout -k 10 120 python tools/bs_stamps.py > gpurun_out/dev/stamps.log 2>&1 || exit 1
fi

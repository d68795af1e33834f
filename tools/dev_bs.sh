#!/bin/bash
# Development cycle for the bucket sort: parity, fusion tests, A/B of the built
# variants, phase stamps.  tools/dev_bs.sh <out-dir> <lib>...
set -o pipefail
out=$1; shift
mkdir -p $out
timeout -k 10 120 python tools/jsdebug.py 64 > $out/jsdbg.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 1
REPS=3 tools/ab.sh "$@" > $out/ab.log 2>&1 || exit 1
if [ -f qpp-fusion-rag_amd/qppfuse/libqppfuse_stamps.so ]; then
  timeout -k 10 120 python tools/bs_stamps.py > $out/stamps.log 2>&1 || exit 1
fi

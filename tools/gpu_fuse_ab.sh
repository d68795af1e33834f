#!/bin/bash
# fusion GPU tests with the current library, then the per-kernel + microbench A/B
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fuse.log 2>&1 || { tail -30 gpurun_out/pytest_fuse.log; exit 1; }
tail -1 gpurun_out/pytest_fuse.log
REPS=${REPS:-3} bash tools/gpu_ab2.sh

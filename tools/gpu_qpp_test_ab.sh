#!/bin/bash
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_qpp.py tests/test_gpu_boundary.py tests/test_gpu_learned.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qpp.log 2>&1 || { tail -30 gpurun_out/pytest_qpp.log; exit 1; }
tail -1 gpurun_out/pytest_qpp.log
bash tools/gpu_qpp_ab.sh

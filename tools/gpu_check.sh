#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 trace + PMC passes.
# Every GPU step has its own time limit; steps chained so the first failure ends the call.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
cat $O/bench.log
bash tools/profile.sh $O/prof
echo all-done

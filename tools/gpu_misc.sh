#!/bin/bash
# Box pass: workspace-path A/B + stamps, the writer A/B (mmap vs pwrite), e2e with timers.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
bash tools/gpu_xl_ab.sh
for i in 1 2; do
  timeout -k 10 120 python -u tools/writebench.py
  QFIO_WRITE_PWRITE=1 timeout -k 10 120 python -u tools/writebench.py
done
QFIO_TIMING=1 timeout -k 10 300 python -u tools/e2e.py > gpurun_out/e2e_t.json 2> gpurun_out/e2e_t.err || { tail -20 gpurun_out/e2e_t.err; exit 1; }
grep -v "^\[qfio\]   " gpurun_out/e2e_t.err | tail -40
cat gpurun_out/e2e_t.json

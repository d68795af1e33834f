#!/bin/bash
# Round-4 pass O: host loader after the false-sharing fixes and the streamed dedupe —
# load_runs phase times (QFIO_TIMING) and the file-to-file e2e on the GPU box's host.
set -e
O=gpurun_out/r04o
mkdir -p $O
QFIO_TIMING=1 timeout -k 10 300 python -u tools/prof_load_runs.py > $O/load_runs_phases.txt 2>&1 || { tail -30 $O/load_runs_phases.txt; exit 1; }
grep "load_runs\|parse \|intern docno\|dedupe\|sort distinct\|  ranks\|hash+part" $O/load_runs_phases.txt | head -24
timeout -k 10 300 python -u tools/e2e.py --repeat 3 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
tail -1 $O/e2e.json

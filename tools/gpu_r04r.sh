#!/bin/bash
# Round-4 pass R: the host loader at HEAD — load_runs phases, file-to-file e2e, the
# 03_qpp stage (raw .res -> .qpp through qfio_read_score_lists)
set -e
O=gpurun_out/r04r
mkdir -p $O
QFIO_TIMING=1 timeout -k 10 300 python -u tools/prof_load_runs.py > $O/load_runs_phases.txt 2>&1 || { tail -30 $O/load_runs_phases.txt; exit 1; }
grep "^load_runs" $O/load_runs_phases.txt
timeout -k 10 300 python -u tools/e2e.py --repeat 3 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
tail -1 $O/e2e.json
timeout -k 10 300 python -u tools/e2e.py --qpp --repeat 3 > $O/e2e_qpp.json 2> $O/e2e_qpp.err || { tail -30 $O/e2e_qpp.err; exit 1; }
tail -1 $O/e2e_qpp.json

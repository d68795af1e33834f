#!/bin/bash
# Round-4 pass C: what the bucket sort's LDS bank conflicts cost.  Development builds
# that stop after the count (stop2) or the scatter (stop4), each also with timing-only
# probes that make the count atomics (PROBE_CNT) and / or the scatter stores
# (PROBE_SCAT) conflict-free — wrong results, same instruction stream.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04c
mkdir -p $O
REPS=2 bash tools/ab_kernels.sh tools/ab/lib_stop2.so tools/ab/lib_stop2c.so tools/ab/lib_stop4.so tools/ab/lib_stop4s.so tools/ab/lib_stop4cs.so > $O/ab_conflict.txt 2>&1 || { tail -20 $O/ab_conflict.txt; exit 1; }
cat $O/ab_conflict.txt
echo r04c-done

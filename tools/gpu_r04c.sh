#!/bin/bash
# Round-4 pass C: (1) what the bucket sort's LDS bank conflicts cost — development
# builds that stop after the count (stop2) or the scatter (stop4), also with
# timing-only probes that make the count atomics (PROBE_CNT) and / or the scatter
# stores (PROBE_SCAT) conflict-free (wrong results, same instruction stream);
# (2) the join's phase costs (tools/gpu_join_phases.sh); (3) min-max with
# non-temporal loads.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04c
mkdir -p $O
REPS=2 bash tools/ab_kernels.sh tools/ab/lib_stop2.so tools/ab/lib_stop2c.so tools/ab/lib_stop4.so tools/ab/lib_stop4s.so tools/ab/lib_stop4cs.so > $O/ab_conflict.txt 2>&1 || { tail -20 $O/ab_conflict.txt; exit 1; }
cat $O/ab_conflict.txt
JPH_OUT=$O/jph bash tools/gpu_join_phases.sh > $O/join_phases.txt 2>&1 || { tail -20 $O/join_phases.txt; exit 1; }
cat $O/join_phases.txt
for i in 1 2; do
  for L in qpp-fusion-rag_amd/qppfuse/libqppfuse.so tools/ab/lib_mmnt.so; do
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py > $O/micro_$(basename $L .so)_$i.json 2>&1 || { tail -20 $O/micro_$(basename $L .so)_$i.json; exit 1; }
    echo "$(basename $L) $(cat $O/micro_$(basename $L .so)_$i.json | tail -1)"
  done
done
echo r04c-done

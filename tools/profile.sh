#!/bin/bash
# rocprofv3 passes over a short bench run (run from the repo root on the GPU box).
# 1: kernel trace + stats; 2: FETCH_SIZE; 3: WRITE_SIZE (separate passes, gfx950 TCC slots);
# 4: SQ_INSTS_VALU + SQ_WAVES (the VALU issue roof of the fusion kernels).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${1:-gpurun_out/prof}
ARGS="--steps 10 --warmup 2 --cpu-sample 0 --native-sample 0 --check 0"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/valu -o run -- python3 bench.py $ARGS > $OUT/bench_valu.log 2>&1
echo profile-done

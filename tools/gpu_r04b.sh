#!/bin/bash
# Round-4 GPU pass B: parity suite on the current library, then learned fusion
# (C5) A/B — separate join + docid-tie sort kernels (lib_chain) against the one
# join_learned_kernel (current) — and the C5 / C2 bench lines.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
cp qpp-fusion-rag_amd/qppfuse/libqppfuse.so tools/ab/lib_cur.so
FUSEBENCH_METHODS=learned REPS=3 bash tools/ab_kernels.sh tools/ab/lib_chain.so tools/ab/lib_cur.so > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
timeout -k 10 300 python -u bench.py --workload c5 --warmup 5 --steps 20 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -30 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -30 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
echo all-done

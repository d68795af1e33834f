#!/bin/bash
# Round-4 GPU pass B (the measurement pass): parity suite + smoke, the bench lines of
# every config, the C2 steady state, rocprofv3 kernel trace + PMC passes of the C2
# bench (tools/profile.sh), SQ counters, an A/B of the last sort change, end to end.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --warmup 50 --steps 400 --cpu-sample 0 --native-sample 0 > $O/bench_c2_steady.json 2> $O/bench_c2_steady.err || { tail -30 $O/bench_c2_steady.err; exit 1; }
for w in c1 c4 c5 c3; do
  timeout -k 10 400 python -u bench.py --workload $w --warmup 5 --steps 20 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -30 $O/bench_$w.err; exit 1; }
  echo "$w: $(python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])")"
done
bash tools/profile.sh $O/prof > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
SQPMC_OUT=$O/sqpmc bash tools/gpu_sqpmc.sh > $O/sqpmc.txt 2>&1 || { tail -30 $O/sqpmc.txt; exit 1; }
REPS=2 bash tools/ab_kernels.sh tools/ab/lib_stop2.so tools/ab/lib_stop2c.so tools/ab/lib_stop4.so tools/ab/lib_stop4s.so tools/ab/lib_stop4cs.so > $O/ab_conflict.txt 2>&1 || { tail -20 $O/ab_conflict.txt; exit 1; }
cat $O/ab_conflict.txt
timeout -k 10 300 python -u tools/e2e.py --repeat 3 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
cat $O/e2e.json
echo all-done

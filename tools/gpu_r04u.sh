#!/bin/bash
# Round-4 pass U (measurement at HEAD: one-wave C1 workgroups, host loader): GPU suite + smoke, the default bench line,
# the C2 steady state, every config's line, rocprofv3 kernel trace + PMC passes
# (tools/profile.sh), SQ counters, the weights-only normalise A/B, end to end.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --warmup 50 --steps 400 --cpu-sample 0 --native-sample 0 > $O/bench_c2_steady.json 2> $O/bench_c2_steady.err || { tail -30 $O/bench_c2_steady.err; exit 1; }
for w in c1 c4 c5 c3; do
  timeout -k 10 400 python -u bench.py --workload $w --warmup 5 --steps 20 > $O/bench_$w.json 2> $O/bench_$w.err || { tail -30 $O/bench_$w.err; exit 1; }
  echo "$w: $(python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_ms'])")"
done
bash tools/profile.sh $O/prof > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
SQPMC_OUT=$O/sqpmc bash tools/gpu_sqpmc.sh > $O/sqpmc.txt 2>&1 || { tail -30 $O/sqpmc.txt; exit 1; }
timeout -k 10 300 python -u tools/e2e.py --repeat 3 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
cat $O/e2e.json
bash tools/gpu_r04q.sh
echo all-done

#!/bin/bash
# Round-4 pass G: GPU suite at HEAD (one-launch learned weights, LDS-image GBDT),
# C5 bench lines, kernel stats of C5, copy-probe shapes (fewer workgroups per CU,
# one-shot grid).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c5_$i.json 2> $O/c5_$i.err || { tail -30 $O/c5_$i.err; exit 1; }
  echo "c5 $(python3 -c "import json; d=json.load(open('$O/c5_$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5prof -o run -- python3 bench.py --workload c5 --steps 10 --warmup 2 --cpu-sample 0 --native-sample 0 --check 0 > $O/c5prof.log 2>&1 || { tail -30 $O/c5prof.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/c5prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
timeout -k 10 120 ./tools/copy_probe 1073741824 probe2 > $O/copy_probe2.jsonl 2>&1 || { tail -5 $O/copy_probe2.jsonl; exit 1; }
cat $O/copy_probe2.jsonl
echo r04g-done

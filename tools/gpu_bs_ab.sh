#!/bin/bash
# Bucket-sort A/B on one box: parity tests of the fusion path, then the C2 fuse
# timings alternating QF_JS_BLOCK=12 (bucket_sort_kernel) and 14 (bsort_kernel),
# then rocprofv3 kernel stats + SQ_INSTS_VALU of the six-method launch for each.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/bsab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
  for B in 12 14; do
    echo -n "JS=$B: "
    QF_JS_BLOCK=$B timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith('fuse:')})"
  done
done
for B in 12 14; do
  QF_JS_BLOCK=$B timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$B -o run -- python3 tools/fusebench.py > $O/k$B.log 2>&1
  QF_JS_BLOCK=$B timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/v$B -o run -- python3 tools/fusebench.py > $O/v$B.log 2>&1
  python3 - $O $B <<'PY'
import csv, glob, sys, collections
O, B = sys.argv[1], sys.argv[2]
f = glob.glob(f'{O}/k{B}/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'qf::' in r['Name']: print('  k%s %-55s %8.1f us x%s' % (B, r['Name'][:55], float(r['AverageNs'])/1e3, r['Calls']))
f = glob.glob(f'{O}/v{B}/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'qf::' in r['Kernel_Name']: acc[(r['Kernel_Name'][:40], r['Counter_Name'])].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()): print('  v%s %-40s %-14s %.3e' % (B, k[0], k[1], sum(v)/len(v)))
PY
done
echo ab-done

#!/bin/bash
# Per-phase VALU of bsort_kernel: development builds that stop after phase n
# (-DQF_BS_STOP=n: 1 range, 2 count, 3 scan, 4 scatter, 5 rank) and the full one,
# each under rocprofv3 (SQ_INSTS_VALU + kernel time) on the C2 six-method launch.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/bsph
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_learned.py tests/test_gpu_fusion.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for n in 1 2 3 4 5 full; do
  if [ $n = full ]; then L=qpp-fusion-rag_amd/qppfuse/libqppfuse.so; else L=qpp-fusion-rag_amd/qppfuse/libqppfuse_stop$n.so; fi
  QF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/v$n -o run -- python3 tools/fusebench.py > $O/v$n.log 2>&1
  QF_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$n -o run -- python3 tools/fusebench.py > $O/k$n.log 2>&1
  python3 - $O $n <<'PY'
import csv, glob, sys, collections
O, n = sys.argv[1], sys.argv[2]
f = glob.glob(f'{O}/k{n}/**/run_kernel_stats.csv', recursive=True)[0]
t = {r['Name'][:30]: float(r['AverageNs'])/1e3 for r in csv.DictReader(open(f)) if 'bsort' in r['Name']}
f = glob.glob(f'{O}/v{n}/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'bsort' in r['Kernel_Name']: acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(n, {k: round(v, 1) for k, v in t.items()}, {k: '%.4e' % (sum(v)/len(v)) for k, v in acc.items()})
PY
done
echo phases-done

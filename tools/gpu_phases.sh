#!/bin/bash
# Per-phase VALU + time of one kernel: tools/gpu_phases.sh <kernel substring> <lib> [<lib> ...]
# (development builds that stop after a phase; each lib under rocprofv3: SQ_INSTS_VALU
# and kernel time of the C2 six-method qf_fuse launch, tools/fusebench.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
K=$1; shift
O=gpurun_out/ph_$K
mkdir -p $O
for L in "$@"; do
  n=$(basename $L .so)
  QF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/v$n -o run -- python3 tools/fusebench.py > $O/v$n.log 2>&1
  QF_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$n -o run -- python3 tools/fusebench.py > $O/k$n.log 2>&1
  python3 - $O $n $K <<'PY'
import csv, glob, sys, collections
O, n, K = sys.argv[1], sys.argv[2], sys.argv[3]
f = glob.glob(f'{O}/k{n}/**/run_kernel_stats.csv', recursive=True)[0]
t = {r['Name'][:40]: round(float(r['AverageNs'])/1e3, 1) for r in csv.DictReader(open(f)) if K in r['Name']}
f = glob.glob(f'{O}/v{n}/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if K in r['Kernel_Name']: acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(n, t, {k: '%.4e' % (sum(v)/len(v)) for k, v in acc.items()})
PY
done
echo phases-done

#!/bin/bash
# Per-phase cost of the LDS join (join_kernel, C2 six-method launch of
# tools/fusebench.py): development builds tools/ab/lib_jstop<n>.so that stop after
# phase n (-DQF_JOIN_STOP=n: 1 loads + table init, 2 hash insert, 3 first-seen
# numbering, 4 group offsets / slot words, 5 placement; full = + ordered sums and
# stores), each under rocprofv3 — kernel time and one --pmc pass of SQ counters.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=${JPH_OUT:-gpurun_out/jph}
mkdir -p $O
for n in 1 2 3 4 5 full; do
  if [ $n = full ]; then L=qpp-fusion-rag_amd/qppfuse/libqppfuse.so; else L=tools/ab/lib_jstop$n.so; fi
  QF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU --kernel-trace --output-format csv -d $O/v$n -o run -- python3 tools/fusebench.py > $O/v$n.log 2>&1
  QF_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$n -o run -- python3 tools/fusebench.py > $O/k$n.log 2>&1
  python3 - $O $n <<'PY'
import csv, glob, sys, collections
O, n = sys.argv[1], sys.argv[2]
f = glob.glob(f'{O}/k{n}/**/run_kernel_stats.csv', recursive=True)[0]
t = {r['Name'][:30]: round(float(r['AverageNs'])/1e3, 1) for r in csv.DictReader(open(f)) if 'JoinCfg' in r['Name']}
f = glob.glob(f'{O}/v{n}/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'JoinCfg' in r['Kernel_Name']: acc[r['Counter_Name']].append(float(r['Counter_Value']))
print(n, t, {k: '%.4e' % (sum(v)/len(v)) for k, v in sorted(acc.items())}, flush=True)
PY
done
echo join-phases-done

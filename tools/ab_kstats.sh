#!/bin/bash
# Per-kernel rocprofv3 stats of the C2 six-method qf_fuse launch for each library:
# tools/ab_kstats.sh <libA> <libB> ...  (summary lines on stdout)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for L in "$@"; do
  n=$(basename $L .so)
  QF_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/$n -o run -- python3 tools/fusebench.py > gpurun_out/abk_$n.log 2>&1
  echo "== $n"
  python3 -c "
import csv,glob
f=glob.glob('gpurun_out/abk/$n/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'qf::' in r['Name']: print('  %-60s %8.1f us x%s' % (r['Name'][:60], float(r['AverageNs'])/1e3, r['Calls']))
"
done

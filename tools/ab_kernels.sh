#!/bin/bash
# A/B of libraries by per-kernel time (rocprofv3 kernel stats of tools/fusebench.py),
# alternating REPS times: tools/ab_kernels.sh <libA> <libB> [...]
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/abk2
mkdir -p $O
for i in $(seq ${REPS:-3}); do
  for L in "$@"; do
    n=$(basename $L .so)_$i
    QF_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 tools/fusebench.py > $O/$n.log 2>&1
    python3 - $O $n <<'PY'
import csv, glob, sys
O, n = sys.argv[1], sys.argv[2]
f = glob.glob(f'{O}/{n}/**/run_kernel_stats.csv', recursive=True)[0]
import re; dg = re.findall(r"ok ([0-9a-f]{16})", open(f"{O}/{n}.log").read()); print(n, dg, {r['Name'].split('(')[0].split('::')[-1][:22]: round(float(r['AverageNs'])/1e3, 1)
          for r in csv.DictReader(open(f)) if 'sort' in r['Name'] or 'join' in r['Name']})
PY
  done
done

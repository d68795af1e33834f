#!/bin/bash
# Round-4 pass F: the LDS-staged GBDT walk (tools/ab/lib_gbdt.so): learned-fusion GPU
# tests through it, C5 bench A/B against HEAD's library, C5 kernel stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04f
mkdir -p $O
QPPFUSE_LIB=tools/ab/lib_gbdt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_learned.py -x -v --timeout 120 --timeout-method thread > $O/pytest_learned.log 2>&1 || { tail -60 $O/pytest_learned.log; exit 1; }
tail -2 $O/pytest_learned.log
for i in 1 2 3; do
  for L in qpp-fusion-rag_amd/qppfuse/libqppfuse.so tools/ab/lib_gbdt.so; do
    n=$(basename $L .so)
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c5 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c5_${n}_$i.json 2> $O/c5_${n}_$i.err || { tail -30 $O/c5_${n}_$i.err; exit 1; }
    echo "c5 $n $(python3 -c "import json; d=json.load(open('$O/c5_${n}_$i.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done
QPPFUSE_LIB=tools/ab/lib_gbdt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5prof -o run -- python3 bench.py --workload c5 --steps 10 --warmup 2 --cpu-sample 0 --native-sample 0 --check 0 > $O/c5prof.log 2>&1 || { tail -30 $O/c5prof.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/c5prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1))
PY
echo r04f-done

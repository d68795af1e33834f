#!/bin/bash
# SQ counters of the C2 six-method qf_fuse kernels (tools/fusebench.py): VALU / LDS
# instruction counts, LDS array cycles, bank conflicts, LDS issue stalls, wave cycles.
# Usage: tools/gpu_sqpmc.sh [lib]   (one rocprofv3 --pmc pass; <= 8 SQ counters)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=${SQPMC_OUT:-gpurun_out/sqpmc}
mkdir -p $O
L=${1:-qpp-fusion-rag_amd/qppfuse/libqppfuse.so}
QF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/p1 -o run -- python3 tools/fusebench.py > $O/p1.log 2>&1
QF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-trace --output-format csv -d $O/p2 -o run -- python3 tools/fusebench.py > $O/p2.log 2>&1
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for d in ("p1", "p2"):
    f = glob.glob(f'{O}/{d}/**/run_counter_collection.csv', recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'qf::' in r['Kernel_Name']:
            acc[(r['Kernel_Name'].split('(')[0][-28:], r['Counter_Name'])].append(float(r['Counter_Value']))
    for k, v in sorted(acc.items()): print('%-30s %-22s %.4e' % (k[0], k[1], sum(v) / len(v)))
PY
echo sqpmc-done

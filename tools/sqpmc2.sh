#!/bin/bash
# SQ counter passes over tools/fusebench.py (kernel trace only).
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${1:-gpurun_out/sq2}
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
i=1
for P in "$P1" "$P2"; do
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/fusebench.py > $OUT/p$i.log 2>&1 || exit $?
  i=$((i+1))
done

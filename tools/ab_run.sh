#!/bin/bash
# One A/B driver for development builds, alternating libraries on one box (replaces
# round 4's per-pass gpu_r04*.sh scripts).
#   tools/ab_run.sh MODE OUT LIB1 [LIB2 ...]
# MODE kstats: rocprofv3 --kernel-trace --stats of tools/fusebench.py (the C2 six-method
#              qf_fuse launch, repeated) -> per-kernel average us + the outputs' digest
#      pmc:    one --pmc pass (SQ_INSTS_VALU / SALU / LDS, bank conflicts) of the same
#      kbench: rocprofv3 --kernel-trace --stats of bench.py (BENCH_ARGS appended) -> every
#              qf kernel's average us (the QPP / min-max kernels included)
#      bench:  bench.py (default C2 line; BENCH_ARGS appended) -> ms/step, qf_fuse ms, parity
# Env: REPS (3), FUSEBENCH_METHODS / FUSEBENCH_SYNTH (tools/fusebench.py), BENCH_ARGS.
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -e
MODE=$1; OUT=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
for i in $(seq ${REPS:-3}); do
  for L in "$@"; do
    n=$(basename "$L" .so)_$i
    case $MODE in
      kstats)
        QF_LIB=$L timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/$n" -o run -- python3 tools/fusebench.py > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
        python3 tools/ab_summary.py kstats "$OUT/$n" "$OUT/$n.log" ;;
      pmc)
        QF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
          SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace --output-format csv \
          -d "$OUT/$n" -o run -- python3 tools/fusebench.py > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
        python3 tools/ab_summary.py pmc "$OUT/$n" "$OUT/$n.log" ;;
      kbench)
        QPPFUSE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/$n" -o run -- python3 bench.py --warmup 2 --steps 10 --cpu-sample 0 \
          --native-sample 0 --check 0 --ndcg-sample 0 $BENCH_ARGS > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
        python3 tools/ab_summary.py kbench "$OUT/$n" "$OUT/$n.log" ;;
      bench)
        QPPFUSE_LIB=$L timeout -k 10 300 python3 -u bench.py --warmup 5 --steps 20 --cpu-sample 0 \
          --native-sample 0 $BENCH_ARGS > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
        python3 tools/ab_summary.py bench "$OUT/$n.json" ;;
      *) echo "unknown mode $MODE"; exit 2 ;;
    esac
  done
done

#!/bin/bash
# A/B of qf_fuse paths on C2 (development): bench (fast, no CPU legs) for each
# QF_JS_BLOCK value given, then one rocprofv3 kernel-stats run of the first.
set -o pipefail
out=gpurun_out/ab_js
mkdir -p $out
for b in "$@"; do
  QF_JS_BLOCK=$b timeout -k 10 120 python bench.py --cpu-sample 0 --ndcg-sample 0 --steps 50 > $out/b_$b.json 2> $out/b_$b.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
QF_JS_BLOCK=$1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --ndcg-sample 0 --steps 20 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || exit 1

#!/bin/bash
# A/B of builds on one box, every kernel of tools/microbench.py: REPS=3 tools/ab_all.sh <libA> <libB> ...
set -e
for i in $(seq ${REPS:-3}); do
  for L in "$@"; do
    echo -n "$(basename $L): "
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('minmax', 'qpp_raw', 'colminmax', 'normalize', 'fuse:rrf', 'fuse:combsum+combmnz+rrf+wcombsum+wcombmnz+wrrf')})"
  done
done

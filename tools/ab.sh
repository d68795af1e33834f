#!/bin/bash
# A/B of builds on the same box, alternating: REPS=3 tools/ab.sh <libA> <libB> [<libC> ...]
# (QF_JS_BLOCK etc. pass through; prints the fuse timings of tools/microbench.py)
set -e
for i in $(seq ${REPS:-3}); do
  for L in "$@"; do
    echo -n "$(basename $L): "
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith('fuse:combsum+') or k.startswith('fuse:rrf')})"
  done
done

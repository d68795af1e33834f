#!/bin/bash
# A/B of two builds on the same box, alternating: tools/ab.sh <libA> <libB> [reps]
# (QF_JS_BLOCK etc. pass through; prints the fuse timings of tools/microbench.py)
set -e
for i in $(seq ${3:-3}); do
  for L in "$1" "$2"; do
    echo -n "$(basename $L): "
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith('fuse:combsum+') or k.startswith('fuse:rrf')})"
  done
done

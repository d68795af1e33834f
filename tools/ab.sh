#!/bin/bash
# A/B of two builds on the same box: tools/ab.sh <libA> <libB> (alternating runs)
set -e
for i in 1 2; do
  for L in "$1" "$2"; do
    echo -n "$(basename $L): "
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith('fuse') or k=='qpp_raw'})"
  done
done

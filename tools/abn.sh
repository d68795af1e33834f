#!/bin/bash
# microbench fuse timings for several builds: tools/abn.sh lib1 lib2 ...
for L in "$@"; do
  echo -n "$(basename $L): "
  QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k[5:]: d[k] for k in d if k.startswith('fuse')})"
done

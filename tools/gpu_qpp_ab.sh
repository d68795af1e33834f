#!/bin/bash
# QPP kernel: phase stamps of the stamps build + alternating microbench timings of two builds
set -e
timeout -k 10 120 python3 tools/qpp_stamps.py
for i in 1 2 3; do
  for L in qpp-fusion-rag_amd/qppfuse/ab/libA.so qpp-fusion-rag_amd/qppfuse/ab/libB.so; do
    echo -n "$(basename $L): "
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('minmax','qpp_raw','colminmax','normalize','fuse:combsum+combmnz+rrf+wcombsum+wcombmnz+wrrf')})"
  done
done

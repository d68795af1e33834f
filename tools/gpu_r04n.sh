#!/bin/bash
# Round-4 pass N: QPP tail divisions through div_int — QPP parity tests, then alternating
# microbench timings of HEAD's build and this one.
set -e
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_qpp.py tests/test_gpu_learned.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for L in tools/ab/lib_qpp_head.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so; do
    echo -n "$i $(basename $L): "
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('qpp_raw','colminmax','normalize')})"
  done
done

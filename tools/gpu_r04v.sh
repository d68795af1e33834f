#!/bin/bash
# Round-4 pass V: min-max with two lists per wavefront for batches <= 32,768 lists —
# norm GPU tests, C1 bench lines and the C2-shaped min-max (17,260 lists of 1,000:
# the sequential branch, as a sharded C2 rank runs it), HEAD's build against this one
set -e
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_norm.py tests/test_gpu_boundary.py tests/test_gpu_fusion.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for L in tools/ab/lib_head.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so; do
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1.json 2> $O/c1.err || { tail -20 $O/c1.err; exit 1; }
    echo "$i $(basename $L) c1 $(python3 -c "import json; d=json.load(open('$O/c1.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
    QF_LIB=$L timeout -k 10 120 python -u tools/microbench.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   c2-shaped', {k: d[k] for k in ('minmax',)})"
  done
done

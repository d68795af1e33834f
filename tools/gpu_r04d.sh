#!/bin/bash
# Round-4 pass D: the GPU suite at HEAD (five-VALU digit match; QPP chains with
# their LDS reads issued ahead and phase C's x_j by readlane), qf_qpp_raw digest +
# time A/B against the build before them (tools/ab/lib_r04base.so), C1 bench A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in 1 2; do
  for L in tools/ab/lib_r04base.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so; do
    n=$(basename $L .so)
    QPPFUSE_LIB=$L timeout -k 10 120 python -u tools/qpp_digest.py > $O/qpp_${n}_$i.json 2> $O/qpp_${n}_$i.err || { tail -30 $O/qpp_${n}_$i.err; exit 1; }
    echo "qpp $n $(cat $O/qpp_${n}_$i.json)"
  done
done
for i in 1 2 3; do
  for L in tools/ab/lib_r04base.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so; do
    n=$(basename $L .so)
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --workload c1 --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c1_${n}_$i.json 2> $O/c1_${n}_$i.err || { tail -30 $O/c1_${n}_$i.err; exit 1; }
    echo "c1 $n $(python3 -c "import json; d=json.load(open('$O/c1_${n}_$i.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
  done
done
for i in 1 2; do
  for L in tools/ab/lib_r04base.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so; do
    n=$(basename $L .so)
    QPPFUSE_LIB=$L timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c2_${n}_$i.json 2> $O/c2_${n}_$i.err || { tail -30 $O/c2_${n}_$i.err; exit 1; }
    echo "c2 $n $(python3 -c "import json; d=json.load(open('$O/c2_${n}_$i.json')); print(d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done
echo r04d-done

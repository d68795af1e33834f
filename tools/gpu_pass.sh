# development pass (round 5): GPU tests of the fusion path, then A/B of the libraries
set -o pipefail
O=${PASS_OUT:-gpurun_out/pass}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
REPS=${REPS:-2} tools/ab_run.sh kstats $O/k tools/ab/lib_base.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so
REPS=1 tools/ab_run.sh pmc $O/p tools/ab/lib_base.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so

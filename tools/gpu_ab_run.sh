set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
REPS=4 timeout -k 10 400 bash tools/ab.sh qpp-fusion-rag_amd/qppfuse/ab/libA.so qpp-fusion-rag_amd/qppfuse/ab/libB.so

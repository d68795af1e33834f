set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 --native-sample 0 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity_vs_oracle'], d.get('ndcg10_delta_vs_ref'))"
REPS=3 bash tools/gpu_ab2.sh

#!/bin/bash
# Round-end evidence on one GPU box: GPU tests, smoke, the default bench line, every
# other BASELINE config's line, the end-to-end drop-in timing and the rocprofv3
# passes.  Each GPU step has its own time limit; the first failure ends the call.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/refresh
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
for w in c1 c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
timeout -k 10 300 python -u tools/e2e.py --repeat 3 > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
# the N > 1 step (sharding, the QPP min/max all-reduce, the pipelined top-k gather)
# rehearsed with two gloo ranks on this box's one GPU
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo \
  --rehearse-one-gpu --steps 20 --warmup 3 > $O/bench_dist2_gloo.json 2> $O/bench_dist2_gloo.err \
  || { tail -20 $O/bench_dist2_gloo.err; exit 1; }
# the workspace path (queries above 10,240 entries) and the LDS path it is priced against
for shape in "500 16 4000" "3452 16 1000" "3452 10 1000"; do
  timeout -k 10 300 python -u tools/xlbench.py $shape >> $O/xl_path.jsonl 2> $O/xl.err || { tail -20 $O/xl.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5prof -o run -- \
  python3 bench.py --workload c5 --steps 20 --warmup 3 --cpu-sample 0 --native-sample 0 --check 0 > $O/c5prof.log 2>&1
bash tools/profile.sh $O/prof
bash tools/gpu_sqpmc.sh > $O/sqpmc.txt
echo refresh-done

#!/bin/bash
# Round-4 GPU pass A: parity suite, copy-ceiling probe, C2 bench, the gloo
# two-rank rehearsal with gather parity, the 03_qpp stage file to file, SQ
# counters and the kernel trace of the bench.  Every GPU step has its own time
# limit; the first failure ends the call.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 60 tools/copy_probe > $O/copy_probe.jsonl 2>&1 || { cat $O/copy_probe.jsonl; exit 1; }
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --rehearse-one-gpu --warmup 5 --steps 20 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -30 $O/bench_gloo2.err; exit 1; }
timeout -k 10 300 python -u tools/e2e.py --qpp --repeat 2 > $O/e2e_qpp.json 2> $O/e2e_qpp.err || { tail -30 $O/e2e_qpp.err; exit 1; }
cat $O/e2e_qpp.json
SQPMC_OUT=$O/sqpmc bash tools/gpu_sqpmc.sh > $O/sqpmc.txt 2>&1 || { tail -30 $O/sqpmc.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-sample 0 --native-sample 0 --check 0 > $O/bench_trace.log 2>&1 || { tail -30 $O/bench_trace.log; exit 1; }
REPS=2 bash tools/ab_kernels.sh tools/ab/lib_base.so tools/ab/lib_chain.so > $O/ab_chain.txt 2>&1 || { tail -20 $O/ab_chain.txt; exit 1; }
cat $O/ab_chain.txt
REPS=2 bash tools/ab_kernels.sh tools/ab/lib_cur.so tools/ab/lib_jsa.so tools/ab/lib_hoist.so tools/ab/lib_clamp.so tools/ab/lib_ntload.so > $O/ab_jsa.txt 2>&1 || { tail -20 $O/ab_jsa.txt; exit 1; }
cat $O/ab_jsa.txt
FUSEBENCH_METHODS=learned REPS=2 bash tools/ab_kernels.sh tools/ab/lib_chain.so tools/ab/lib_cur.so > $O/ab_c5.txt 2>&1 || { tail -20 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
timeout -k 10 300 python -u bench.py --workload c5 --warmup 5 --steps 20 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -30 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
BSPH_OUT=$O/bsph bash tools/gpu_bs_phases.sh > $O/bs_phases.txt 2>&1 || { tail -20 $O/bs_phases.txt; exit 1; }
cat $O/bs_phases.txt
echo all-done

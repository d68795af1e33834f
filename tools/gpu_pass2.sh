set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_synth.py tests/test_gpu_fusion.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/c2.json 2> $O/c2.err || { tail -30 $O/c2.err; exit 1; }
python3 tools/ab_summary.py bench $O/c2.json
python3 -c "import json; d=json.load(open('$O/c2.json')); print(d['ndcg10'], d.get('ndcg10_delta_vs_ref'), d['parity_vs_oracle'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --warmup 2 --steps 5 --cpu-sample 0 --native-sample 0 --ndcg-sample 0 --check 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/r05d/prof/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)): print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY

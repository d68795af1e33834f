set -e
timeout -k 10 300 python -u tools/e2e.py --dir /tmp/qf_e2e --repeat 1 > gpurun_out/e2e.log 2>&1
timeout -k 10 300 python -u -c "
import sys, time, cProfile, pstats
sys.path[:0] = ['qpp-fusion-rag_amd', '.']
from qppfuse import fusion
cProfile.run(\"runs = fusion.load_runs('/tmp/qf_e2e')\", '/tmp/lr.prof')
pstats.Stats('/tmp/lr.prof').sort_stats('tottime').print_stats(12)
" > gpurun_out/lr_prof.txt 2>&1
tail -1 gpurun_out/e2e.log

#!/bin/bash
# Round-4 pass H: non-temporal join loads A/B (tools/ab/lib_joinnt.so vs lib_head.so),
# the default bench line with the one-shot copy ceiling.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04h
mkdir -p $O
REPS=3 bash tools/ab_kernels.sh tools/ab/lib_head.so tools/ab/lib_joinnt.so > $O/ab_joinnt.txt 2>&1 || { tail -20 $O/ab_joinnt.txt; exit 1; }
cat $O/ab_joinnt.txt
timeout -k 10 300 python -u bench.py --warmup 5 --steps 20 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['copy_ceiling_gbs'], r['frac_of_copy_ceiling'])"
echo r04h-done

#!/bin/bash
# Round-4 pass L: QPP weights inside the fusion (qf_fuse_qpp), raw-QPP learned weights
# (bench.py C2 / C4 / C5 A/B: HEAD~ = tools/ab/lib_head.so with the old bench step is
# not comparable, so the A/B is the step itself: this tree vs the parity test), GPU
# QPP + fusion tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for w in c2 c4 c5; do
    timeout -k 10 300 python -u bench.py --workload $w --warmup 5 --steps 20 --cpu-sample 0 --native-sample 0 > $O/${w}_$i.json 2> $O/${w}_$i.err || { tail -30 $O/${w}_$i.err; exit 1; }
    echo "$w $(python3 -c "import json; d=json.load(open('$O/${w}_$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_oracle'])")"
  done
done
echo r04l-done

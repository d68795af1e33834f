#!/bin/bash
# A/B of development knobs read from the environment (one library): rocprofv3 kernel
# stats of tools/fusebench.py under each setting, reported as µs per qf_fuse call
# (every fusion kernel's total time / the 5 calls) — chunked launches included.
#   tools/ab_env.sh OUT 'ENV=..' 'ENV=..' ...   ('-' = no knob); REPS (2), FUSEBENCH_SYNTH
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
for i in $(seq ${REPS:-2}); do
  k=0
  for E in "$@"; do
    k=$((k + 1)); n=cfg${k}_$i
    if [ "$E" = "-" ]; then E=""; fi
    env $E timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/$n" -o run -- python3 tools/fusebench.py > "$OUT/$n.log" 2>&1 || { tail -20 "$OUT/$n.log"; exit 1; }
    python3 - "$OUT/$n" "$OUT/$n.log" "$E" <<'PY'
import csv, glob, re, sys
f = glob.glob(f"{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
dg = re.findall(r"ok ([0-9a-f]{16})", open(sys.argv[2]).read())
t, tot = {}, 0.0
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("sort", "join", "fuse_large")):
        us = float(r["TotalDurationNs"]) / 1e3 / 5  # fusebench: 5 qf_fuse calls
        t[re.sub(r"^(void )?qf::", "", r["Name"].split("(")[0])[:40]] = round(us, 1)
        tot += us
print(sys.argv[3] or "default", dg, round(tot, 1), t, flush=True)
PY
  done
done

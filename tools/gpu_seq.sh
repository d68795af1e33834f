# Run GPU steps in order, each under its own time limit; an ordinary failure (exit 1,
# e.g. a failing test) goes on to the next step, anything else (a fault, an abort, a
# time limit, a signal) ends the sequence.  Each argument is one step:
#   bash tools/gpu_seq.sh 'SECONDS command ...' 'SECONDS command ...'
# Output: gpurun_out/seq/<n>.log per step; the exit code is the worst one seen.
set -o pipefail
mkdir -p gpurun_out/seq
worst=0
n=0
for step in "$@"; do
  n=$((n + 1))
  secs=${step%% *}
  cmd=${step#* }
  echo "[seq $n] ${secs}s: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > gpurun_out/seq/$n.log 2>&1
  rc=$?
  echo "[seq $n] rc=$rc"
  tail -4 gpurun_out/seq/$n.log
  if [ $rc -gt $worst ]; then worst=$rc; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[seq] stopping after step $n (rc=$rc)"
    exit $rc
  fi
done
exit $worst

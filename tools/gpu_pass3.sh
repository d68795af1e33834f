# A/B of the big-union sort configurations on SURVEY §8(d)'s C2 (kstats + pmc)
set -o pipefail
O=${PASS_OUT:-gpurun_out/r05f}; mkdir -p $O
L="qpp-fusion-rag_amd/qppfuse/libqppfuse.so tools/ab/lib_big1.so tools/ab/lib_big2.so tools/ab/lib_big3.so"
FUSEBENCH_SYNTH=nq REPS=2 tools/ab_run.sh kstats $O/k $L || exit 1
FUSEBENCH_SYNTH=nq REPS=1 tools/ab_run.sh pmc $O/p $L || exit 1

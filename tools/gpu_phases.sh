# Phase costs of bsort_fast_kernel from development stop builds (tools/ab/lib_stop<n>.so,
# -DQF_STOP_AT=n: 21 loads + key constants, 22 count, 23 scan, 24 scatter, 25 rank) and the
# library: rocprofv3 time and one --pmc pass each; FUSEBENCH_SYNTH picks the generator.
set -o pipefail
O=${PASS_OUT:-gpurun_out/phases}
mkdir -p $O
LIBS="tools/ab/lib_stop21.so tools/ab/lib_stop22.so tools/ab/lib_stop23.so tools/ab/lib_stop24.so tools/ab/lib_stop25.so qpp-fusion-rag_amd/qppfuse/libqppfuse.so"
REPS=1 tools/ab_run.sh kstats $O/k $LIBS || exit 1
REPS=1 tools/ab_run.sh pmc $O/p $LIBS || exit 1

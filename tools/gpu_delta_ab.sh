#!/bin/bash
# bucket-sort delta shift A/B: rocprof stats on seeded random weights (fusebench) and
# alternating microbench timings with QPP weights
set -e
L=qpp-fusion-rag_amd/qppfuse/ab
bash tools/ab_kstats.sh $L/libD12.so $L/libD16.so $L/libD20.so
REPS=2 timeout -k 10 400 bash tools/ab.sh $L/libD12.so $L/libD16.so $L/libD20.so

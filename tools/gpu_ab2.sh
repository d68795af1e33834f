#!/bin/bash
# A/B of two builds: per-kernel rocprof stats (seeded fusebench) + alternating microbench
set -e
A=qpp-fusion-rag_amd/qppfuse/ab/libA.so; B=qpp-fusion-rag_amd/qppfuse/ab/libB.so
bash tools/ab_kstats.sh $A $B
REPS=${REPS:-3} timeout -k 10 400 bash tools/ab.sh $A $B

#!/bin/bash
# Round-4 pass P: e2e with HEAD~'s loader library and this one, alternated (the fuse
# stage's time moved 0.10 -> 0.19 s between the two e2e records)
set -e
O=gpurun_out/r04p
mkdir -p $O
for i in 1 2; do
  for L in tools/ab/libqfio_old.so qpp-fusion-rag_amd/qppfuse/libqfio.so; do
    QPPFUSE_IO_LIB=$L timeout -k 10 300 python -u tools/e2e.py --repeat 3 > $O/e2e_$i_$(basename $L .so).json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
    echo "$i $(basename $L): $(tail -1 $O/e2e_$i_$(basename $L .so).json)"
  done
done

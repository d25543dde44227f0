#!/bin/bash
# Ramped pieces (1 MiB, 2 MiB, then the wave's piece) for large PUT batches (lab knob).
set -o pipefail
out=gpurun_out/r4r
mkdir -p $out
LAB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for n in 512 256; do
  for r in 0 1024 512; do
    MXEC_LIB=$LAB MXEC_PIPE_RAMP_KB=$r timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned \
        > $out/e2e_${n}_r${r}.json 2> $out/e2e_${n}_r${r}.err || exit 1
  done
done

#!/bin/bash
# 2D piece copies (lab knob) for large PUT batches with digests.
set -o pipefail
out=gpurun_out/r4d
mkdir -p $out
LAB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for n in 512 256 128; do
  for c in 0 1; do
    MXEC_LIB=$LAB MXEC_PIPE_COPY2D=$c timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned \
        > $out/e2e_${n}_2d${c}.json 2> $out/e2e_${n}_2d${c}.err || exit 1
  done
done

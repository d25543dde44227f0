#!/bin/bash
# GET from host memory at 128 / 512 objects: copy modes (auto = waves for
# reconstruct batches; sdma).
set -o pipefail
out=gpurun_out/r4gm
mkdir -p $out
for n in 512 128; do
  for mode in sdma waves; do
    MXEC_PIPE_COPY=$mode timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned --get \
        > $out/e2e_${n}_$mode.json 2> $out/e2e_${n}_$mode.err || exit 1
  done
done

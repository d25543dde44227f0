#!/bin/bash
# GET side from host memory at 128 / 256 / 512 objects (two erasures each),
# without and with verification.
set -o pipefail
out=gpurun_out/r4g
mkdir -p $out
for n in 128 256 512; do
  timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned --get > $out/e2e_$n.json 2> $out/e2e_$n.err || exit 1
done

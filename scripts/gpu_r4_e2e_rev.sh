#!/bin/bash
# Table copies back on the launch streams, adaptive pieces kept: the default
# bench's host legs, then PUT with digests at 128 / 256 / 512 objects.
set -o pipefail
out=gpurun_out/r4e7
mkdir -p $out
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err &&
for n in 128 256 512; do
  timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned > $out/e2e_$n.json 2> $out/e2e_$n.err || exit 1
done

#!/bin/bash
# PUT with digests: piece size 1 / 2 / 4 MiB / whole chunks at 128 and 512 objects.
set -o pipefail
out=gpurun_out/r4e5
mkdir -p $out
for n in 512 128; do
  for p in 1 2 4 0; do
    MXEC_PIPE_PIECE_MB=$p timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned \
        > $out/e2e_${n}_p${p}.json 2> $out/e2e_${n}_p${p}.err || exit 1
  done
done

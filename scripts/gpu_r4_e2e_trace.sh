#!/bin/bash
# PUT with digests at 512 objects: per-piece trace (lab build) and copy modes.
set -o pipefail
out=gpurun_out/r4e2
mkdir -p $out
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_PIPE_TRACE=1 timeout -k 10 400 python -u tools/e2e_bench.py --objects 512 --reps 2 \
    --alloc mxec --modes pinned > $out/e2e_512_trace.json 2> $out/e2e_512_trace.err &&
MXEC_PIPE_COPY=waves timeout -k 10 400 python -u tools/e2e_bench.py --objects 512 --reps 3 --alloc mxec --modes pinned \
    > $out/e2e_512_waves.json 2> $out/e2e_512_waves.err &&
timeout -k 10 400 python -u tools/e2e_bench.py --objects 256 --reps 3 --alloc mxec --modes pinned \
    > $out/e2e_256.json 2> $out/e2e_256.err

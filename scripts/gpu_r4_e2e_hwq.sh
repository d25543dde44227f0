#!/bin/bash
# PUT with digests at 512 objects: do the uploads share a hardware queue with
# the SHA-256 stream?  Copy streams at the highest priority (lab), compute
# streams at the highest priority (lab), and 8 hardware queues per process.
set -o pipefail
out=gpurun_out/r4e4
mkdir -p $out
LAB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
MXEC_LIB=$LAB MXEC_PIPE_TRACE=1 MXEC_PIPE_COPY_PRIO=1 timeout -k 10 400 python -u tools/e2e_bench.py --objects 512 --reps 2 \
    --alloc mxec --modes pinned > $out/prio1.json 2> $out/prio1.err &&
MXEC_LIB=$LAB MXEC_PIPE_TRACE=1 MXEC_PIPE_COPY_PRIO=2 timeout -k 10 400 python -u tools/e2e_bench.py --objects 512 --reps 2 \
    --alloc mxec --modes pinned > $out/prio2.json 2> $out/prio2.err &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/e2e_bench.py --objects 512 --reps 2 \
    --alloc mxec --modes pinned > $out/hwq8.json 2> $out/hwq8.err

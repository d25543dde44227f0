#!/bin/bash
# Table copies on the upload stream: the pipeline tests, then PUT with
# digests at 128 / 256 / 512 objects (trace at 512), then the default bench.
set -o pipefail
out=gpurun_out/r4e3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_storage_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_pipeline.log 2>&1 &&
tail -2 $out/pytest_pipeline.log &&
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so MXEC_PIPE_TRACE=1 timeout -k 10 400 python -u tools/e2e_bench.py --objects 512 --reps 2 \
    --alloc mxec --modes pinned > $out/e2e_512_trace.json 2> $out/e2e_512_trace.err &&
timeout -k 10 400 python -u tools/e2e_bench.py --objects 256 --reps 3 --alloc mxec --modes pinned > $out/e2e_256.json 2> $out/e2e_256.err &&
timeout -k 10 400 python -u tools/e2e_bench.py --objects 128 --reps 3 --alloc mxec --modes pinned > $out/e2e_128.json 2> $out/e2e_128.err &&
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err

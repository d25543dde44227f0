#!/bin/bash
# Adaptive piece size: pipeline tests, PUT with digests at 128 / 256 / 512
# objects, then the default bench line.
set -o pipefail
out=gpurun_out/r4e6
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_storage_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_pipeline.log 2>&1 &&
tail -2 $out/pytest_pipeline.log &&
for n in 128 256 512; do
  timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned > $out/e2e_$n.json 2> $out/e2e_$n.err || exit 1
done &&
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err

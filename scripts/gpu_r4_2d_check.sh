#!/bin/bash
# 2D piece copies on by default in PUT piece waves: pipeline tests, e2e at
# 128 / 256 / 512 objects, two default bench lines in fresh processes.
set -o pipefail
out=gpurun_out/r4d3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_storage_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_pipeline.log 2>&1 &&
tail -1 $out/pytest_pipeline.log &&
for n in 128 256 512; do
  timeout -k 10 300 python -u tools/e2e_bench.py --objects $n --reps 3 --alloc mxec --modes pinned > $out/e2e_$n.json 2> $out/e2e_$n.err || exit 1
done &&
timeout -k 10 600 python bench.py > $out/bench_a.json 2> $out/bench_a.err &&
timeout -k 10 600 python bench.py > $out/bench_b.json 2> $out/bench_b.err

#!/bin/bash
# Body-digest GPU tests + bench line + kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_digest_gpu.py -x -q > gpurun_out/digest.log 2>&1 || { tail -30 gpurun_out/digest.log; exit 1; }
tail -2 gpurun_out/digest.log
timeout -k 10 600 python bench.py --config sums --steps 5 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_sums.json 2> gpurun_out/bench_sums.err || { tail -20 gpurun_out/bench_sums.err; exit 1; }
cat gpurun_out/bench_sums.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sums -o run --output-format csv -- python bench.py --config sums --objects 256 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_sums.log 2>&1 || { tail -20 gpurun_out/prof_sums.log; exit 1; }

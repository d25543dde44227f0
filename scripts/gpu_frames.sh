#!/bin/bash
# Frames + body digests: bench lines and a kernel trace of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in frames sums; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline'], d['cpu_baseline'], d['cpu_baseline_all_cores'], d['spot_check_vs_oracle'], d['extra'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_frames -o run --output-format csv -- python bench.py --config frames --objects 64 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_frames.log 2>&1 || { tail -20 gpurun_out/prof_frames.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sums -o run --output-format csv -- python bench.py --config sums --objects 256 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_sums.log 2>&1 || { tail -20 gpurun_out/prof_sums.log; exit 1; }

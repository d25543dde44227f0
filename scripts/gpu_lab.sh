#!/bin/bash
# Kernel lab + bench + rocprofv3 of the bench command (one GPU session).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
echo "== lab"; timeout -k 10 600 tools/kernel_lab 1024 > gpurun_out/lab.jsonl 2> gpurun_out/lab.err || { cat gpurun_out/lab.err; exit 1; }
cat gpurun_out/lab.jsonl
echo "== bench --extra"; timeout -k 10 900 python bench.py --extra > gpurun_out/bench_extra.json 2> gpurun_out/bench_extra.err || { tail gpurun_out/bench_extra.err; exit 1; }
cat gpurun_out/bench_extra.json
echo "== bench"; timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprofv3 (same bench command)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof2" -o run --output-format csv -- python3 "$R/bench.py" > "$R/gpurun_out/prof2_bench.json" 2> "$R/gpurun_out/prof2_bench.err" || exit 1
cat "$R/gpurun_out/prof2_bench.json"
echo "== rocprofv3 --pmc (HBM traffic, separate passes)"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit 1
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 > "$R/gpurun_out/pmc_write.log" 2>&1 || exit 1
ls "$R/gpurun_out/pmc_fetch" "$R/gpurun_out/pmc_write"

#!/bin/bash
# Config 5 host/device split: enqueue-time probe, then a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/cfg5_probe.py > gpurun_out/cfg5_probe.log 2>&1 || { tail -20 gpurun_out/cfg5_probe.log; exit 1; }
cat gpurun_out/cfg5_probe.log | grep -v amdgpu.ids
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python bench.py --config 5 --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/prof5.log 2>&1 || { tail -20 gpurun_out/prof5.log; exit 1; }
find gpurun_out/prof5 -name "*stats*" | head

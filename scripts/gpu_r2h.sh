#!/bin/bash
# Config 3c under rocprofv3 --kernel-trace: kernel durations and the gaps
# between them (where a step's time goes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); O=gpurun_out/r2h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p3c -o run --output-format csv -- python3 "$R/bench.py" --config 3c --workers 8 --steps 3 --warmup 1 --cpu-seconds 0 > "$R/$O/bench3c.json" 2> "$R/$O/bench3c.err" || { tail "$R/$O/bench3c.err"; exit 1; }
find /tmp/p3c -name "*kernel_stats.csv" -exec cp {} "$R/$O/kernel_stats.csv" \;
find /tmp/p3c -name "*kernel_trace.csv" -exec cp {} "$R/$O/kernel_trace.csv" \;
head -8 "$R/$O/kernel_stats.csv" | cut -c1-200

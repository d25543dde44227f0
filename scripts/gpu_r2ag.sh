#!/bin/bash
# Config 5 (mixed stream): per-class breakdown, the bench line with exact
# algorithmic bytes, and a kernel trace of the same command (GPU busy time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2ag; mkdir -p $O
timeout -k 10 300 python tools/cfg5_breakdown.py > $O/breakdown.jsonl 2> $O/breakdown.err || { tail -20 $O/breakdown.err; exit 1; }
cat $O/breakdown.jsonl
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-extra > $O/bench5.json 2> $O/bench5.err || { tail $O/bench5.err; exit 1; }
cut -c1-400 $O/bench5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r2ag -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 10 --warmup 2 --no-extra --cpu-seconds 0 > "$R/$O/bench5_rocprof.json" 2> "$R/$O/bench5_rocprof.err" || { tail -5 "$R/$O/bench5_rocprof.err"; exit 1; }
find /tmp/r2ag -name "*kernel_trace.csv" -exec cp {} "$R/$O/kernel_trace.csv" \;

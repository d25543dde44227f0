#!/bin/bash
# Config 5 timeline: kernel trace of a few steps (launch count, busy vs idle).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2r; mkdir -p $O
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --cpu-seconds 0 --no-extra > $O/cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg5.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r2r -o run --output-format csv -- python3 "$R/bench.py" --config 5 --steps 4 --warmup 1 --cpu-seconds 0 --no-extra > "$R/$O/cfg5_prof.json" 2> "$R/$O/cfg5_prof.err" || { tail -5 "$R/$O/cfg5_prof.err"; exit 1; }
find /tmp/r2r -name "*kernel_trace.csv" -exec cp {} "$R/$O/cfg5_trace.csv" \;
find /tmp/r2r -name "*kernel_stats.csv" -exec cp {} "$R/$O/cfg5_stats.csv" \;

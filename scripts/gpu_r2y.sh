#!/bin/bash
# Config 3c: callers' speculative decodes queued before the combined launch's
# digest copy -- do they now run beside the hash?  Trace + plain bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2y; mkdir -p $O
MXEC_COMBINE_LOG=1 timeout -k 10 300 python bench.py --config 3c --workers 8 --steps 8 --warmup 2 --cpu-seconds 0 > $O/cfg3c.json 2> $O/cfg3c.err || { tail -20 $O/cfg3c.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3c.json')); r=d['roofline']; print('3c', d['value'], d['ms_per_step'], r['frac'])"
grep "mxec combine" $O/cfg3c.err | tail -4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r2y -o run --output-format csv -- python3 "$R/bench.py" --config 3c --workers 8 --steps 3 --warmup 1 --cpu-seconds 0 > "$R/$O/cfg3c_t.json" 2> "$R/$O/cfg3c_t.err" || { tail -5 "$R/$O/cfg3c_t.err"; exit 1; }
find /tmp/r2y -name "*kernel_trace.csv" -exec cp {} "$R/$O/trace.csv" \;

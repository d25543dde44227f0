#!/bin/bash
# New combiner dependency test; PMC HBM traffic of the current RS kernel
# (configs 2 and ns, --no-extra, FETCH_SIZE / WRITE_SIZE passes); the default
# bench under rocprofv3 --kernel-trace with the per-shape trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2o; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_concurrency_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for cfg in 2 ns; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex rs_apply_fast -d "/tmp/pmc_${cfg}_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --cpu-seconds 0 --no-extra > "$R/$O/pmc_${cfg}_$c.log" 2>&1 || { tail -5 "$R/$O/pmc_${cfg}_$c.log"; exit 1; }
    find "/tmp/pmc_${cfg}_$c" -name "*counter_collection.csv" -exec cp {} "$R/$O/pmc_${cfg}_$c.csv" \;
  done
done
echo "== rocprof default bench (trace)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r2o_def -o run --output-format csv -- python3 "$R/bench.py" > "$R/$O/bench_rocprof.json" 2> "$R/$O/bench_rocprof.err" || { tail -5 "$R/$O/bench_rocprof.err"; exit 1; }
find /tmp/r2o_def -name "*kernel_stats.csv" -exec cp {} "$R/$O/default_kernel_stats.csv" \;
find /tmp/r2o_def -name "*kernel_trace.csv" -exec cp {} "$R/$O/default_kernel_trace.csv" \;
cd "$R"
python tools/trace_summary.py $O/default_kernel_trace.csv --match rs_apply_fast --out $O/default_trace_summary.json | cut -c1-200
python -c "import json; d=json.load(open('$O/bench_rocprof.json')); print(d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"

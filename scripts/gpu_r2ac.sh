#!/bin/bash
# Device async verify + the GPU suite, then the default bench (object-major
# layout, speculative rebuild) for the round-2 evidence.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2ac; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline'].get('frac_of_box_stream'))
e=d['extra']; print('ns', e['ns']['GiBps_payload'], e['ns']['roofline']['frac'], e['ns']['roofline'].get('frac_of_box_stream')); print('3', e['config3']['GiBps_payload'], e['config3']['ms_per_call']); print('3c', e['config3c']['GiBps_payload'], e['config3c']['ms_per_step'], e['config3c']['roofline']['frac']); print(e['calibration'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/r2ac -o run --output-format csv -- python3 "$R/bench.py" > "$R/$O/bench_rocprof.json" 2> "$R/$O/bench_rocprof.err" || { tail -5 "$R/$O/bench_rocprof.err"; exit 1; }
find /tmp/r2ac -name "*kernel_stats.csv" -exec cp {} "$R/$O/kernel_stats.csv" \;
find /tmp/r2ac -name "*kernel_trace.csv" -exec cp {} "$R/$O/kernel_trace.csv" \;
cd "$R"
python -c "import json; d=json.load(open('$O/bench_rocprof.json')); print('rocprof run', d['value'], d['roofline']['ms_per_launch'])"

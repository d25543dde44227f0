#!/bin/bash
# Round evidence in one GPU call: full -m gpu suite, smoke, the default bench
# line, and rocprofv3 --kernel-trace --stats of the same bench command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/round
mkdir -p $O
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo "== bench"; timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
echo "== rocprofv3 (same bench command)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run --output-format csv -- python3 "$R/bench.py" > "$R/$O/prof_bench.json" 2> "$R/$O/prof_bench.err" || { tail "$R/$O/prof_bench.err"; exit 1; }
cat "$R/$O/prof_bench.json"
find "$R/$O/prof" -name "*kernel_stats.csv" | head -3

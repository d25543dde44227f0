#!/bin/bash
# The auto copy mode as the default: the GPU suite, smoke, the default bench,
# and the lab bench without CU masks (MXEC_PIPE_COPY_CUS=0) for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4m}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
MXEC_PIPE_COPY_CUS=0 MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so timeout -k 10 400 python bench.py --cpu-seconds 1 \
  > "$O/bench_nomask.json" 2> "$O/bench_nomask.err" || { tail -20 "$O/bench_nomask.err"; exit 1; }
echo done

#!/bin/bash
# Round 4 GET-stall study, one call: the copy-mode test, the default bench with
# CU-wave copies (MXEC_PIPE_COPY=waves) and with SDMA after a 10 s pause, and
# tools/host_copy_lab.py.  Each step under its own limit; the first failure ends.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4h}
mkdir -p "$O"
export TMPDIR=/tmp
LAB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -k "copy_modes" -x -v --timeout 200 --timeout-method thread \
  > "$O/pytest_copy_modes.log" 2>&1 || { tail -30 "$O/pytest_copy_modes.log"; exit 1; }
tail -2 "$O/pytest_copy_modes.log"
MXEC_PIPE_COPY=waves MXEC_LIB=$LAB MXEC_PIPE_TRACE=1 timeout -k 10 400 python bench.py --cpu-seconds 1 \
  > "$O/bench_waves.json" 2> "$O/bench_waves.err" || { tail -20 "$O/bench_waves.err"; exit 1; }
BENCH_GET_AFTER_SLEEP=10 MXEC_LIB=$LAB MXEC_PIPE_TRACE=1 timeout -k 10 400 python bench.py --cpu-seconds 1 \
  > "$O/bench_sleep10.json" 2> "$O/bench_sleep10.err" || { tail -20 "$O/bench_sleep10.err"; exit 1; }
timeout -k 10 300 python tools/host_copy_lab.py > "$O/host_copy_lab.jsonl" 2> "$O/host_copy_lab.err" \
  || { tail -20 "$O/host_copy_lab.err"; exit 1; }
# back-to-back processes: the headline right after a process that freed ~64 GB,
# then again after a 30 s pause (is "slow mode" the driver clearing freed VRAM?)
timeout -k 10 200 python bench.py --no-extra --no-e2e --cpu-seconds 0 > "$O/bench_b2b_1.json" 2> "$O/bench_b2b_1.err" || exit 1
sleep 30
timeout -k 10 200 python bench.py --no-extra --no-e2e --cpu-seconds 0 > "$O/bench_b2b_2.json" 2> "$O/bench_b2b_2.err" || exit 1
echo done

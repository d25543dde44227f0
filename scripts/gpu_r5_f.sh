#!/bin/bash
# Round 5: expected digests in one staged copy per wave; the SDMA watch on
# the verified GET read against forced SDMA / waves; the driver's bench; then
# (last: it may fault at exit) the profiler-exit probe without the watch's
# timing events.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5f}
mkdir -p $out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_get_groups_gpu.py \
  tests/test_pipeline_2d_gpu.py tests/test_pipeline_gpu.py tests/test_contract_gpu.py tests/test_storage_gpu.py \
  tests/test_storage_drivers_gpu.py > $out/pytest_sel.log 2>&1 || { tail -30 $out/pytest_sel.log; exit 1; }
tail -1 $out/pytest_sel.log
timeout -k 10 300 python -u tools/watch_diag.py > $out/watch_diag.jsonl 2> $out/watch_diag.err || { tail -5 $out/watch_diag.err; exit 1; }
cat $out/watch_diag.jsonl
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err \
  || { tail -20 $out/bench.err; exit 1; }
cd /tmp
MXEC_PIPE_SDMA_FLOOR=0 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ex_b -o run --output-format csv \
  -- python3 $R/tools/exit_probe.py host_pageable > $R/$out/exit_pageable_floor0.out 2> $R/$out/exit_pageable_floor0.err
echo "{\"what\": \"host_pageable, MXEC_PIPE_SDMA_FLOOR=0\", \"rc\": $?}" | tee -a $R/$out/exit_probe3.jsonl

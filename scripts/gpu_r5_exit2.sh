#!/bin/bash
# The profiler-exit fault follows a host-batch call (profiles/r5/exit_probe.jsonl).
# Which part: the context's teardown (--no-close keeps it), or the watch's
# timing events (MXEC_PIPE_SDMA_FLOOR=0 creates none).  Stops at the first
# run that does not exit 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5x}
mkdir -p $out
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ex_a -o run --output-format csv \
  -- python3 $R/tools/exit_probe.py host_pageable --no-close > $R/$out/exit_pageable_noclose.out 2> $R/$out/exit_pageable_noclose.err
rc=$?; echo "{\"what\": \"host_pageable --no-close\", \"rc\": $rc}" | tee -a $R/$out/exit_probe2.jsonl
[ $rc = 0 ] || exit 1
MXEC_PIPE_SDMA_FLOOR=0 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ex_b -o run --output-format csv \
  -- python3 $R/tools/exit_probe.py host_pageable > $R/$out/exit_pageable_floor0.out 2> $R/$out/exit_pageable_floor0.err
rc=$?; echo "{\"what\": \"host_pageable, MXEC_PIPE_SDMA_FLOOR=0\", \"rc\": $rc}" | tee -a $R/$out/exit_probe2.jsonl
[ $rc = 0 ] || exit 1
echo done

#!/bin/bash
# rocprofv3 --kernel-trace --memory-copy-trace exit fault: which library step
# trips it (tools/exit_probe.py).  The series stops at the first run that
# does not exit 0 (nothing more runs on the GPU after a fault); the order
# goes from the least library work to the most.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5x}
mkdir -p $out
export TMPDIR=/tmp
R=$PWD
for w in "open" "hash" "device" "host_pageable" "host_pinned --no-close" "host_pinned"; do
  tag=$(echo $w | tr ' ' '_')
  ( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ex_$tag -o run --output-format csv \
      -- python3 $R/tools/exit_probe.py $w > $R/$out/exit_$tag.out 2> $R/$out/exit_$tag.err ); rc=$?
  echo "{\"what\": \"$w\", \"rc\": $rc}" | tee -a $out/exit_probe.jsonl
  [ $rc = 0 ] || exit 1
done
echo done

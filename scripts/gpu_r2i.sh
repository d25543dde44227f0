#!/bin/bash
# Wave placement of persistent grids after an HBM kernel; stream-form repeats
# with 1 / 4 waves per workgroup and 1024 / 2048 waves after an HBM kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2i; mkdir -p $O
timeout -k 5 120 tools/sha_stream_lab place > $O/place.jsonl 2>&1 || { cat $O/place.jsonl; exit 1; }
cat $O/place.jsonl
for v in "LAB_FORM=4" "LAB_FORM=3 LAB_WAVES=2048" "LAB_FORM=4 LAB_WAVES=2048"; do
  echo "== $v"
  env $v LAB_BETWEEN=1 timeout -k 5 120 tools/sha_stream_lab repeat > $O/rep.jsonl 2>&1 || { cat $O/rep.jsonl; exit 1; }
  cut -c1-90 $O/rep.jsonl | tr '\n' ' '; echo
done

#!/bin/bash
# Small-chunk encode: whole chunks vs a short last chunk, 8+4 and 4+2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2ah; mkdir -p $O
for km in 8,4 4,2; do
  timeout -k 10 300 python tools/small_chunk_lab.py --km $km > $O/lab_$km.jsonl 2> $O/lab_$km.err || { tail -20 $O/lab_$km.err; exit 1; }
  cat $O/lab_$km.jsonl
done

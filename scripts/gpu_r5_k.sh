#!/bin/bash
# Round 5: plain SDMA copy rates before and after one large HBM free.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5k}
mkdir -p $out
for g in 60 20; do
timeout -k 10 120 python -u tools/sdma_after_free.py --free-gb $g --seconds 8 > $out/after_free_$g.jsonl 2> $out/after_free_$g.err \
  || { tail -5 $out/after_free_$g.err; exit 1; }
tail -1 $out/after_free_$g.jsonl
done

#!/bin/bash
# Round 5: downloads by waves with the copy streams CU-masked away from the
# compute streams (lab build), fresh and right after a 60 GB free.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5n}
mkdir -p $out
export MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for c in 0 60; do
timeout -k 10 500 python -u tools/watch_diag.py --objects 128,512 --kinds put_sha,put_rs,rs,verified --modes sdma,sdma_down_waves,sdma_down_waves_cus16 --reps 3 --churn-each $c \
  > $out/cus_churn$c.jsonl 2> $out/cus_churn$c.err || { tail -5 $out/cus_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/cus_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']])
"
done

#!/bin/bash
# Round 5: downloads by CU waves with uploads by SDMA (lab build), fresh and
# right after 60 GB of HBM is freed, against both engines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5j}
mkdir -p $out
export MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_lab.so
for c in 0 60; do
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds rs,verified,put_rs,put_sha --modes sdma,waves,sdma_down_waves --reps 3 --churn-each $c \
  > $out/split_churn$c.jsonl 2> $out/split_churn$c.err || { tail -5 $out/split_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/split_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']])
"
done

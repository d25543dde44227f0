#!/bin/bash
# Round 5: the final copy policy, every host call kind at 128 / 512 objects,
# healthy and right after a 60 GB HBM free.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5ag}
mkdir -p $out
for c in 0 60; do
timeout -k 10 500 python -u tools/watch_diag.py --objects 128,512 --kinds verified,rs,put_sha,put_rs --modes auto,sdma --reps 3 --churn-each $c \
  > $out/final_churn$c.jsonl 2> $out/final_churn$c.err || { tail -5 $out/final_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/final_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']])
"
done

#!/bin/bash
# Round 5: plain SDMA copy rates before / after one large HBM free; the
# download watch's tests; auto against sdma / waves after a 60 GB free.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5l}
mkdir -p $out
if [ -n "$AFTER_FREE" ]; then
timeout -k 10 120 python -u tools/sdma_after_free.py --free-gb 60 --seconds 8 > $out/after_free_60.jsonl 2> $out/after_free_60.err \
  || { tail -5 $out/after_free_60.err; exit 1; }
tail -1 $out/after_free_60.jsonl
fi
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pipeline_2d_gpu.py \
  > $out/pytest_2d.log 2>&1 || { tail -30 $out/pytest_2d.log; exit 1; }
tail -1 $out/pytest_2d.log
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds rs,verified,put_rs,put_sha --modes auto,sdma --reps 3 --churn-each 60 \
  > $out/auto_churn60.jsonl 2> $out/auto_churn60.err || { tail -5 $out/auto_churn60.err; exit 1; }
python3 -c "
import json
for l in open('$out/auto_churn60.jsonl'):
    r=json.loads(l); print(r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']], [(c.get('sdma_slow'), c.get('sdma_down_slow'), c.get('sdma_down_last_mbps')) for c in r['calls']])
"

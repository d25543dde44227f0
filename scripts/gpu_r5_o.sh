#!/bin/bash
# Round 5: the per-kind engine policy (verified GET downloads by waves, an
# RS-only GET's downloads watched against twice the floor, PUT downloads by
# SDMA unbracketed): pipeline tests, then auto against sdma / waves fresh
# and right after a 60 GB free.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5o}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pipeline_2d_gpu.py \
  tests/test_pipeline_gpu.py tests/test_get_groups_gpu.py > $out/pytest_pipe.log 2>&1 || { tail -30 $out/pytest_pipe.log; exit 1; }
tail -1 $out/pytest_pipe.log
for c in 0 60; do
timeout -k 10 500 python -u tools/watch_diag.py --objects 128,512 --kinds put_sha,put_rs,rs,verified --modes auto,sdma,waves --reps 3 --churn-each $c \
  > $out/policy_churn$c.jsonl 2> $out/policy_churn$c.err || { tail -5 $out/policy_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/policy_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']], [(c['sdma_slow'], c['sdma_down_slow'], c['sdma_down_last_mbps']) for c in r['calls']])
"
done

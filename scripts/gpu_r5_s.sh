#!/bin/bash
# Round 5: verification groups chosen per wave, earlier groups' downloads by
# SDMA and the last group's by waves: tests, then the verified GET at 128 /
# 512 objects fresh and right after a 60 GB free.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5s}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_get_groups_gpu.py \
  tests/test_pipeline_2d_gpu.py tests/test_pipeline_gpu.py tests/test_contract_gpu.py > $out/pytest_pipe.log 2>&1 || { tail -30 $out/pytest_pipe.log; exit 1; }
tail -1 $out/pytest_pipe.log
for c in 0 60; do
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds verified,rs --modes auto,sdma --reps 3 --churn-each $c \
  > $out/vg_churn$c.jsonl 2> $out/vg_churn$c.err || { tail -5 $out/vg_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/vg_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['objects'], r['kind'], r['mode'], r['median_s'], [c['s'] for c in r['calls']], [(c['verify_groups'] if 'verify_groups' in c else None) for c in r['calls']])
"
done

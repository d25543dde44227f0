#!/bin/bash
# Round 5: brackets judged only when their DMAs average >= 1 MiB (pipeline
# tests, the host kinds fresh and after a 74 GB free); the SHA-256 quad form
# alone with and without its K + W ring's barriers / schedule.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r5y}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_pipeline_2d_gpu.py \
  tests/test_pipeline_gpu.py tests/test_get_groups_gpu.py > $out/pytest_pipe.log 2>&1 || { tail -30 $out/pytest_pipe.log; exit 1; }
tail -1 $out/pytest_pipe.log
for c in 0 74; do
timeout -k 10 400 python -u tools/watch_diag.py --objects 128,512 --kinds put_sha,put_rs,rs,verified --modes auto --reps 3 --churn $c \
  > $out/kinds_churn$c.jsonl 2> $out/kinds_churn$c.err || { tail -5 $out/kinds_churn$c.err; exit 1; }
python3 -c "
import json
for l in open('$out/kinds_churn$c.jsonl'):
    r=json.loads(l); print('churn$c', r['objects'], r['kind'], r['median_s'], [(c['s'], c['sdma_slow'], c['sdma_down_slow'], c['wave_blocks']) for c in r['calls']])
"
done
for lib in lab lab_nosync lab_nosched; do
MXEC_LIB=$PWD/maxio_amd/lib/libmaxio_ec_$lib.so timeout -k 10 200 python -u tools/sha_alone.py >> $out/sha_alone.jsonl 2> $out/sha_alone_$lib.err \
  || { tail -5 $out/sha_alone_$lib.err; exit 1; }
done
cat $out/sha_alone.jsonl

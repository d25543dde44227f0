#!/bin/bash
# Round 2: stream-form SHA-256.  New GPU tests first (stream form forced and
# chosen), then the whole suite, then config 3c / 3 / 3c-12 benches and the
# kernel alone (kernel_lab) on the big batches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=gpurun_out/r2d
mkdir -p $O
echo "== stream tests"
timeout -k 10 400 python -u -m pytest tests/test_sha_stream_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -5 $O/pytest_stream.log
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for c in "3c --workers 8" "3" "3c --workers 12" "3c --workers 4"; do
  tag=$(echo $c | tr -d ' -')
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 0 > $O/cfg$tag.json 2> $O/cfg$tag.err || { tail -20 $O/cfg$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg$tag.json')); print('$c', d['value'], d['ms_per_step'], d['spot_check_vs_oracle'], d.get('extra'))"
done

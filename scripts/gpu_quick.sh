#!/bin/bash
# GPU tests, then bench configs 2 and 5 (no CPU leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-2 5}; do
  echo "== config $c"
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/bench_cfg$c.json 2> gpurun_out/bench_cfg$c.err || { tail -20 gpurun_out/bench_cfg$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_cfg$c.json')); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['spot_check_vs_oracle'])"
done

#!/bin/bash
# Every BASELINE config through bench.py on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 2 3 4a 4b 5; do
  echo "== config $c"
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_cfg$c.json 2> gpurun_out/bench_cfg$c.err || { tail -20 gpurun_out/bench_cfg$c.err; exit 1; }
  cat gpurun_out/bench_cfg$c.json
done

#!/bin/bash
# Mixed-shape batches: the GPU tests that cover grouped RS launches, then
# config 5 with the classes on 4 streams vs one encode + one reconstruct
# batch call per step (grouped launches), alternating, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/mixed; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_mixed_batch_gpu.py tests/test_configs_gpu.py tests/test_cut_tiles_gpu.py tests/test_gpu_parity.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for mode in streams batch; do
    BENCH_MIXED_MODE=$mode timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-extra > $O/cfg5_${mode}_$r.json 2> $O/cfg5_${mode}_$r.err || { tail -20 $O/cfg5_${mode}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/cfg5_${mode}_$r.json')); print('$mode', $r, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['spot_check_vs_oracle'])"
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BENCH_MIXED_MODE=batch timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 3 --warmup 1 --no-extra --cpu-seconds 0 > $R/$O/prof.json 2> $R/$O/prof.err || { tail -5 $R/$O/prof.err; exit 1; }
cat $R/$O/prof.json | head -c 600

#!/bin/bash
# Descriptor tables copied on a side stream (default) vs in the launch
# stream (MXEC_DESC_UPLOAD=inline): full GPU suite, then configs 5 (batch
# calls) and 3c alternating, then a trace of config 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/upload; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for up in inline stream; do
    for c in 5 3c; do
      MXEC_DESC_UPLOAD=$up BENCH_MIXED_MODE=batch timeout -k 10 300 python bench.py --config $c --steps 8 --warmup 2 --no-extra --cpu-seconds 0 > $O/cfg${c}_${up}_$r.json 2> $O/cfg${c}_${up}_$r.err || { tail -20 $O/cfg${c}_${up}_$r.err; exit 1; }
      python -c "import json; d=json.load(open('$O/cfg${c}_${up}_$r.json')); print('$up', '$c', $r, d['value'], d['ms_per_step'], d['spot_check_vs_oracle'] if 'spot_check_vs_oracle' in d else '')"
    done
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
BENCH_MIXED_MODE=batch timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config 5 --steps 3 --warmup 1 --no-extra --cpu-seconds 0 > $R/$O/prof.json 2> $R/$O/prof.err || { tail -5 $R/$O/prof.err; exit 1; }

#!/bin/bash
# Config 5 with its 15 classes on 1 vs 4 streams, alternating, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2s; mkdir -p $O
for r in 1 2 3; do
  for ns in 1 4 8; do
    BENCH_MIXED_STREAMS=$ns timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --cpu-seconds 0 --no-extra > $O/cfg5_s${ns}_$r.json 2> $O/cfg5_s${ns}_$r.err || { tail -20 $O/cfg5_s${ns}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/cfg5_s${ns}_$r.json')); print('round $r streams $ns', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['spot_check_vs_oracle'])"
  done
done

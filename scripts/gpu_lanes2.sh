#!/bin/bash
# Combiner launch lanes (MXEC_COMBINE_STREAMS; a second lane opens only under
# lane_limit) at light and heavy GET load and on the chip-filling config 3c.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lanes2; mkdir -p $O
for L in 1 2; do
  for t in 16 64; do
    MXEC_COMBINE_STREAMS=$L timeout -k 10 300 python tools/e2e_get_bench.py --objects 256 --threads $t --cpu-objects 2 --reps 2 > $O/e2e_t${t}_L$L.json 2> $O/e2e_t${t}_L$L.err || { tail $O/e2e_t${t}_L$L.err; exit 1; }
    python -c "import json; d=json.load(open('$O/e2e_t${t}_L$L.json')); print('L=$L t=$t', 'healthy', d['gpu_healthy']['GiBps'], 'degraded', d['gpu_degraded']['GiBps'], 'put', d['gpu_put']['GiBps'])"
  done
  for c in 3c 3; do
    MXEC_COMBINE_STREAMS=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/cfg${c}_L$L.json 2> $O/cfg${c}_L$L.err || { tail -5 $O/cfg${c}_L$L.err; exit 1; }
    python -c "import json; d=json.load(open('$O/cfg${c}_L$L.json')); print('L=$L cfg $c', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# Combiner lanes (MXEC_COMBINE_STREAMS) 2 / 3 / 4: 8 MiB GETs and PUTs at
# W = 16 and 64, two alternating rounds (tools/e2e_get_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2p; mkdir -p $O
for r in 1 2; do
 for W in 16 64; do
  for L in 2 3 4; do
    MXEC_COMBINE_STREAMS=$L timeout -k 10 240 python tools/e2e_get_bench.py --objects 384 --reps 2 --threads $W --cpu-objects 0 > $O/l${L}_w${W}_$r.json 2> $O/l${L}_w${W}_$r.err || { tail -20 $O/l${L}_w${W}_$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/l${L}_w${W}_$r.json'))
print('round $r W=$W lanes=$L: GET healthy', d['gpu_healthy']['GiBps'], 'degraded', d['gpu_degraded']['GiBps'], 'PUT', d['gpu_put']['GiBps'], 'cores', d['gpu_healthy']['host_cores_busy'])"
  done
 done
done

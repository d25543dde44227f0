#!/bin/bash
# Combiner lanes 2 / 4 against HIP hardware queues 4 (default) / 16
# (GPU_MAX_HW_QUEUES): 8 MiB GET / PUT at W = 16 and 64, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2q; mkdir -p $O
for r in 1 2; do
 for W in 16 64; do
  for Q in 4 16; do
   for L in 2 4; do
    GPU_MAX_HW_QUEUES=$Q MXEC_COMBINE_STREAMS=$L timeout -k 10 240 python tools/e2e_get_bench.py --objects 384 --reps 2 --threads $W --cpu-objects 0 > $O/q${Q}_l${L}_w${W}_$r.json 2> $O/q${Q}_l${L}_w${W}_$r.err || { tail -20 $O/q${Q}_l${L}_w${W}_$r.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/q${Q}_l${L}_w${W}_$r.json'))
print('round $r W=$W hwq=$Q lanes=$L: GET healthy', d['gpu_healthy']['GiBps'], 'degraded', d['gpu_degraded']['GiBps'], 'PUT', d['gpu_put']['GiBps'], 'cores', d['gpu_healthy']['host_cores_busy'])"
   done
  done
 done
done

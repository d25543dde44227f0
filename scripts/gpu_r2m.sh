#!/bin/bash
# single-request crossover at BASELINE configs[0]'s shape
# (one 10 MiB chunk, 2 parity, one shard deleted): GPU path vs the reference
# algorithm on the host cores at W concurrent GETs; combiner lanes 2 vs 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2m; mkdir -p $O
for L in 2 4; do
for W in 1 16 48 128; do
  n=$(( W * 2 )); [ $n -lt 8 ] && n=8; [ $n -gt 256 ] && n=256
  c=$n; [ $c -gt 64 ] && c=64; [ $L = 4 ] && c=0
  MXEC_COMBINE_STREAMS=$L timeout -k 10 300 python tools/e2e_get_bench.py --k 1 --parity 2 --chunk-size 10485760 --erasures 1 --objects $n --reps 1 --threads $W --cpu-objects $c > $O/cfg0_l${L}_w$W.json 2> $O/cfg0_l${L}_w$W.err || { tail -20 $O/cfg0_l${L}_w$W.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/cfg0_l${L}_w$W.json'))
print('lanes=$L W=$W', 'gpu healthy', d['gpu_healthy']['GiBps'], 'degraded', d['gpu_degraded']['GiBps'], 'cpu ref degraded', d.get('cpu_reference_degraded_${W}t', {}).get('GiBps'), 'cpu 1t', d.get('cpu_reference_degraded_1t', {}).get('GiBps'), 'single GET ms', d.get('gpu_healthy_1thread', {}).get('ms_per_object'))"
done
done
for L in 2 4; do
  MXEC_COMBINE_STREAMS=$L timeout -k 10 300 python tools/e2e_get_bench.py --objects 512 --reps 2 --threads 64 --cpu-objects 0 > $O/get8_l$L.json 2> $O/get8_l$L.err || { tail -20 $O/get8_l$L.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/get8_l$L.json'))
print('lanes=$L 8 MiB objects W=64 gpu healthy', d['gpu_healthy']['GiBps'], 'degraded', d['gpu_degraded']['GiBps'], 'put', d['gpu_put']['GiBps'], 'single GET ms', d['gpu_healthy_1thread']['ms_per_object'])"
done

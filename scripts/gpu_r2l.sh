#!/bin/bash
# pinned vs pageable host buffers, three runs each,
# alternating, 64 and 128 request threads (tools/e2e_get_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2l; mkdir -p $O
for t in 64 128; do
 for i in 1 2 3; do
  for mode in pageable pinned; do
    flag=""; [ $mode = pinned ] && flag="--pinned"
    timeout -k 10 240 python tools/e2e_get_bench.py --objects 512 --reps 2 --threads $t --cpu-objects 0 $flag > $O/get_${t}_${mode}_$i.json 2> $O/get_${t}_${mode}_$i.err || { tail -20 $O/get_${t}_${mode}_$i.err; exit 1; }
    python - $O/get_${t}_${mode}_$i.json $t $mode $i <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
g = lambda k: (d.get(k) or {})
print(f"threads={sys.argv[2]} {sys.argv[3]} run {sys.argv[4]}: GET healthy {g('gpu_get')['GiBps'] if 'gpu_get' in d else d.get('gpu_healthy',{}).get('GiBps')} "
      f"({(g('gpu_get') or g('gpu_healthy')).get('host_cores_busy')} cores), degraded {g('gpu_degraded').get('GiBps')}, "
      f"PUT {g('gpu_put').get('GiBps')} ({g('gpu_put').get('host_cores_busy')} cores)", flush=True)
PY
  done
 done
done

#!/bin/bash
# Combiner launch lanes: GPU tests that go through the combiner, then configs
# 3 / 3c and the file-layer GET bench with MXEC_COMBINE_STREAMS=1,2,(3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lanes
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "concurren or combin or storage or reconstruct" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in ${LANES:-1 2 3}; do
  for c in 3 3c; do
    MXEC_COMBINE_STREAMS=$L timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/cfg${c}_L$L.json 2> $O/cfg${c}_L$L.err || { tail -20 $O/cfg${c}_L$L.err; exit 1; }
    python -c "import json; d=json.load(open('$O/cfg${c}_L$L.json')); print('L=$L cfg $c', d['value'], d['ms_per_step'], d['spot_check_vs_oracle'])"
  done
  MXEC_COMBINE_STREAMS=$L timeout -k 10 300 python tools/e2e_get_bench.py --objects 256 --threads 64 --cpu-objects 4 > $O/e2e_L$L.json 2> $O/e2e_L$L.err || { tail $O/e2e_L$L.err; exit 1; }
  echo "L=$L e2e"; cat $O/e2e_L$L.json
done

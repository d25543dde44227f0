#!/bin/bash
# File-layer GET / PUT end to end at several request-thread counts, then the
# SHA-bearing bench configs (regression check of the host-path changes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/getscan; mkdir -p $O
for t in ${THREADS:-16 64 128}; do
  timeout -k 10 300 python tools/e2e_get_bench.py --objects 512 --threads $t --cpu-objects 4 --reps 2 > $O/e2e_t$t.json 2> $O/e2e_t$t.err || { tail $O/e2e_t$t.err; exit 1; }
  echo "threads $t"; cat $O/e2e_t$t.json
done
for c in ${CONFIGS:-3 3c}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 > $O/cfg$c.json 2> $O/cfg$c.err || { tail -20 $O/cfg$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg$c.json')); print('cfg $c', d['value'], d['ms_per_step'], d['spot_check_vs_oracle'])"
done

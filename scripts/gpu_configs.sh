#!/bin/bash
# Every bench config on one GPU (one box, one table), then the file-layer
# PUT / GET end-to-end bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/configs
mkdir -p $O
for c in ${CONFIGS:-2 ns 3 3c 4a 4b 5 sums frames}; do
  echo "== config $c"
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 > $O/bench_cfg$c.json 2> $O/bench_cfg$c.err || { tail -20 $O/bench_cfg$c.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_cfg$c.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_copy_GBps'), (d.get('cpu_baseline') or {}).get('value'), d['spot_check_vs_oracle'])"
done
echo "== e2e files"
timeout -k 10 600 python tools/e2e_get_bench.py --objects 256 --threads 64 > $O/e2e_files_t64.json 2> $O/e2e.err || { tail $O/e2e.err; exit 1; }
cat $O/e2e_files_t64.json

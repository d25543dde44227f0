#!/bin/bash
# Headline with the object-major layout and the larger RS-pattern probe:
# 3 separate processes, then ns once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2aa; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extra > $O/cfg2_$r.json 2> $O/cfg2_$r.err || { tail -20 $O/cfg2_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_$r.json')); r=d['roofline']; print('cfg2 run $r', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_stream_GBps'), r.get('frac_of_box_stream'), d['spot_check_vs_oracle'])"
done
timeout -k 10 300 python bench.py --config ns --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfgns.json 2> $O/cfgns.err || { tail -20 $O/cfgns.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfgns.json')); r=d['roofline']; print('cfg ns', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_stream_GBps'), r.get('frac_of_box_stream'))"

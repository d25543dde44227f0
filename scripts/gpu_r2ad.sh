#!/bin/bash
# Padded object-major encode layout: headline in 3 fresh processes, then
# the default command once.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2ad; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extra > $O/cfg2_$r.json 2> $O/cfg2_$r.err || { tail -20 $O/cfg2_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_$r.json')); r=d['roofline']; print('cfg2 run $r', d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('box_stream'), r.get('box_stream_GBps'), r.get('frac_of_box_stream'), d['spot_check_vs_oracle'])"
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline'].get('frac_of_box_stream'), d['spot_check_vs_oracle'])
e=d['extra']; print('ns', e['ns']['GiBps_payload'], e['ns']['roofline']['frac'], e['ns']['roofline'].get('frac_of_box_stream')); print('3', e['config3']['GiBps_payload'], e['config3']['ms_per_call']); print('3c', e['config3c']['GiBps_payload'], e['config3c']['ms_per_step'], e['config3c']['roofline']['frac']); print('put', e['put_path_encode_plus_sha256'])"

#!/bin/bash
# Host enqueue cost of the headline call, three processes; then the default
# bench (3c extra with 6 timed steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2ae; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python tools/enqueue_probe.py > $O/enq_$r.json 2> $O/enq_$r.err || { tail -20 $O/enq_$r.err; exit 1; }
  cat $O/enq_$r.json | cut -c1-600
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['roofline'].get('frac_of_box_stream'))
e=d['extra']; print('ns', e['ns']['GiBps_payload'], e['ns']['roofline']['frac'], e['ns']['roofline'].get('frac_of_box_stream')); print('3', e['config3']['GiBps_payload'], e['config3']['ms_per_call']); print('3c', e['config3c']['GiBps_payload'], e['config3c']['ms_per_step'], e['config3c']['roofline']['frac'])"

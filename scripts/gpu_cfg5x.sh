#!/bin/bash
# Config 5 inside the default line's extras vs standalone, descriptor upload
# side stream vs inline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/cfg5x; mkdir -p $O
for up in inline default; do
  if [ $up = inline ]; then export MXEC_DESC_UPLOAD=inline; else unset MXEC_DESC_UPLOAD; fi
  timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-extra --cpu-seconds 0 > $O/solo_$up.json 2> $O/solo_$up.err || { tail -20 $O/solo_$up.err; exit 1; }
  python -c "import json; d=json.load(open('$O/solo_$up.json')); print('solo $up', d['value'], d['ms_per_step'])"
  timeout -k 10 500 python bench.py --cpu-seconds 0 > $O/default_$up.json 2> $O/default_$up.err || { tail -20 $O/default_$up.err; exit 1; }
  python -c "import json; d=json.load(open('$O/default_$up.json')); e=d['extra']; print('default $up', d['value'], 'cfg5', e['config5']['GiBps_payload'], e['config5']['ms_per_step'], 'ns', e['ns']['GiBps_payload'])"
done

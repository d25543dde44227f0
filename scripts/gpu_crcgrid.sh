#!/bin/bash
# CRC tile kernel grid (workgroups per CU) on the body-digest config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/crcgrid; mkdir -p $O
for r in 1 2; do
  for b in 8 32 128 512; do
    MXEC_CRC_BPC=$b timeout -k 10 300 python bench.py --config sums --steps 5 --warmup 1 --cpu-seconds 0 > $O/sums_$b_$r.json 2> $O/sums_$b_$r.err || { tail -5 $O/sums_$b_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/sums_$b_$r.json')); print('bpc $b r$r', d['value'], d['ms_per_step'], d['roofline']['achieved'], d.get('spot_check_vs_oracle'), (d.get('extra') or {}).get('breakdown', {}).get('crc32c'))"
  done
done

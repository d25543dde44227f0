#!/bin/bash
# HBM traffic of the dominant RS kernel (configs 2 and ns): two separate
# rocprofv3 --pmc passes per config (FETCH_SIZE, WRITE_SIZE), counters only on
# rs_apply_fast, summarised here by tools/pmc_summary.py (gfx950 FETCH_SIZE
# correction); the raw CSVs are dropped to keep gpurun_out small.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O="$R/gpurun_out/pmc"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-2 ns}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $cfg $c"
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex rs_apply_fast -d "/tmp/pmc/${cfg}_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 2 --warmup 1 --cpu-seconds 0 --no-extra > "$O/${cfg}_$c.log" 2>&1 || { tail -5 "$O/${cfg}_$c.log"; exit 1; }
    find "/tmp/pmc/${cfg}_$c" -name "*counter_collection.csv" -exec cp {} "$O/${cfg}_$c.csv" \;
  done
done
ls -la "$O"

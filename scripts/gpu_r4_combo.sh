#!/bin/bash
# The combiner tests, then the shard-pad placement study (gpu_r4_place5.sh).
set -o pipefail
out=gpurun_out/r4c
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "combin or lone" > $out/pytest_combiner.log 2>&1 &&
tail -3 $out/pytest_combiner.log &&
bash scripts/gpu_r4_place5.sh

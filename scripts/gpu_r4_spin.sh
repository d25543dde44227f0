#!/bin/bash
# Config 3 per-call time: blocking-sync waits (default) vs spin waits.
set -o pipefail
out=gpurun_out/r4s
mkdir -p $out
timeout -k 10 300 python bench.py --config 3 --no-extra > $out/cfg3_block.json 2> $out/cfg3_block.err &&
MXEC_SPIN_WAIT=1 timeout -k 10 300 python bench.py --config 3 --no-extra > $out/cfg3_spin.json 2> $out/cfg3_spin.err &&
timeout -k 10 300 python bench.py --config 3 --no-extra > $out/cfg3_block2.json 2> $out/cfg3_block2.err

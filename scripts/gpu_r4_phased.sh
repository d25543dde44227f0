#!/bin/bash
# Time-divided read / write phases for the RS pattern (tools/phased_lab.py).
set -o pipefail
out=gpurun_out/r4ph
mkdir -p $out
timeout -k 10 300 python -u tools/phased_lab.py --objects 512 > $out/phased.jsonl 2> $out/phased.err

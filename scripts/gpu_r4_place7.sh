#!/bin/bash
# Which half of the RS pattern is slow in a slow placement: reads of the data
# shards only, parity writes only, both; plus a plain read of the same bytes.
set -o pipefail
out=gpurun_out/r4p7
mkdir -p $out
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 6 --free-each --spacer-mib 0,3000,17000,41000,9000,0 \
    --grids 1024 --parts --pads-kib 8256 > $out/parts.jsonl 2> $out/parts.err

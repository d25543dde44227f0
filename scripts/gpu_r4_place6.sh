#!/bin/bash
# Shard stride vs placement, configs[1] (4+2 x 10 MiB) and the north-star
# shape (8+4 x 1 MiB): each allocation timed at several shard pads.
set -o pipefail
out=gpurun_out/r4p6
mkdir -p $out
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 5 --free-each --spacer-mib 0,3000,17000,41000,9000 \
    --grids 1024 --pads-kib 2112,4096,5120,6144,6208,7168,8256 > $out/cfg2_pads_1024.jsonl 2> $out/cfg2_pads_1024.err &&
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 3 --free-each --spacer-mib 0,41000,9000 \
    --grids 256 --pads-kib 2112,4096,6144,8256 > $out/cfg2_pads_256.jsonl 2> $out/cfg2_pads_256.err &&
timeout -k 10 400 python -u tools/placement_lab.py --shape 8,4,1 --objects 4096 --allocs 4 --free-each --spacer-mib 0,3000,17000,41000 \
    --grids 512 --pads-kib 0,64,128,256,512,1024 > $out/ns_pads.jsonl 2> $out/ns_pads.err

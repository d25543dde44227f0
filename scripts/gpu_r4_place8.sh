#!/bin/bash
# The RS pattern's halves at the bench's own layout (pad 2 MiB + 64 KiB) over
# allocations placed several ways: in a slow placement, is it the reads, the
# writes or their mix?
set -o pipefail
out=gpurun_out/r4p8
mkdir -p $out
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 6 --free-each --spacer-mib 0,3000,17000,41000,9000,0 \
    --grids 1024 --parts > $out/parts_default_pad.jsonl 2> $out/parts_default_pad.err &&
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 3 --grids 1024 --parts > $out/parts_kept.jsonl 2> $out/parts_kept.err

#!/bin/bash
# Placement lab at configs[1]'s full batch (1024 objects): three batches kept
# side by side, then six placed one at a time behind spacers of varying size.
set -o pipefail
out=gpurun_out/r4p
mkdir -p $out
timeout -k 10 300 python -u tools/placement_lab.py --objects 1024 --allocs 3 --check > $out/place_kept.jsonl 2> $out/place_kept.err &&
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 6 --free-each \
    --spacer-mib 0,3000,17000,41000,90000,150000 > $out/place_spacers.jsonl 2> $out/place_spacers.err

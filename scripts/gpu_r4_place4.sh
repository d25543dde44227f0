#!/bin/bash
# Grid sweep (workgroups per CU of the uniform RS launch) over full configs[1]
# batches placed several ways: is a smaller grid robust where 1024 is slow?
set -o pipefail
out=gpurun_out/r4p4
mkdir -p $out
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 3 --grids 1024,512,256,128 > $out/grids_kept.jsonl 2> $out/grids_kept.err &&
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 6 --free-each --spacer-mib 0,3000,17000,41000,90000,9000 --grids 1024,512,256,128 > $out/grids_spacers.jsonl 2> $out/grids_spacers.err

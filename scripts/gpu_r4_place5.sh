#!/bin/bash
# Does the shard stride decide a slow placement?  Every allocation times the
# encode with the shards S + pad apart for several pads, inside one buffer.
set -o pipefail
out=gpurun_out/r4p5
mkdir -p $out
P=0,4,64,1024,2112,2048,3072,4160,8256,6144
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 3 --grids 1024 --pads-kib $P --variants "v2=MXEC_RS_VECS:2;v1=MXEC_RS_VECS:1" > $out/pads_kept.jsonl 2> $out/pads_kept.err &&
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 5 --free-each --spacer-mib 0,3000,17000,41000,9000 --grids 1024 --pads-kib $P --variants "v2=MXEC_RS_VECS:2;v1=MXEC_RS_VECS:1" > $out/pads_spacers.jsonl 2> $out/pads_spacers.err

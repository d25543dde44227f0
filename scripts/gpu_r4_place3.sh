#!/bin/bash
# RS schedule variants on full configs[1] batches that land fast and slow:
# which schedule holds up in the slow placements without losing the fast ones?
set -o pipefail
out=gpurun_out/r4p3
mkdir -p $out
V='v2=MXEC_RS_VECS:2;v1=MXEC_RS_VECS:1;v2b2048=MXEC_RS_VECS:2,MXEC_RS_BPC:2048;bpc256=MXEC_RS_BPC:256;bpc2048=MXEC_RS_BPC:2048;st0=MXEC_RS_STORE_NT:0;ld0=MXEC_RS_LOAD_NT:0'
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 3 --grids 1024,512 --variants "$V" --check > $out/variants_a.jsonl 2> $out/variants_a.err &&
timeout -k 10 400 python -u tools/placement_lab.py --objects 1024 --allocs 6 --free-each --spacer-mib 0,3000,17000,41000,90000,9000 --grids 1024 --variants "$V" > $out/variants_b.jsonl 2> $out/variants_b.err

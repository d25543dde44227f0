#!/bin/bash
# Is the first full configs[1] batch slow for good or only because it came
# first?  Three kept batches, then two revisit passes over all three; then the
# same with a 20 s idle before the first allocation is measured.
set -o pipefail
out=gpurun_out/r4p2
mkdir -p $out
timeout -k 10 300 python -u tools/placement_lab.py --objects 1024 --allocs 3 --revisit 2 > $out/place_revisit.jsonl 2> $out/place_revisit.err &&
timeout -k 10 300 python -u tools/placement_lab.py --objects 1024 --allocs 3 --revisit 1 --grids 512,1024 > $out/place_revisit_512.jsonl 2> $out/place_revisit_512.err

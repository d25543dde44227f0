#!/bin/bash
# PUT from host memory with every chunk's SHA-256 at 128 / 512 objects per
# batch: does the chain hide behind the PCIe transfer once enough is in flight?
set -o pipefail
out=gpurun_out/r4e
mkdir -p $out
timeout -k 10 400 python -u tools/e2e_bench.py --objects 128 --reps 3 > $out/e2e_128.json 2> $out/e2e_128.err &&
timeout -k 10 500 python -u tools/e2e_bench.py --objects 512 --reps 3 > $out/e2e_512.json 2> $out/e2e_512.err

#!/bin/bash
# HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, separate passes) of the CRC and
# AES-GCM frame kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in sums frames; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -d "$R/gpurun_out/pmc_${c}_$ctr" -o run --output-format csv -- python3 "$R/bench.py" --config $c --objects 64 --steps 2 --warmup 1 --cpu-seconds 0 > "$R/gpurun_out/pmc_${c}_$ctr.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_${c}_$ctr.log"; exit 1; }
  done
done
cd "$R"
python3 tools/pmc_summary.py gpurun_out/pmc_sums_FETCH_SIZE gpurun_out/pmc_sums_WRITE_SIZE crc_tiles_kernel $((64 * 41943040)) --what "crc_tiles_kernel, bench.py --config sums --objects 64 (64 x 40 MiB bodies); algorithmic = body bytes" --out gpurun_out/pmc_crc.json
python3 tools/pmc_summary.py gpurun_out/pmc_frames_FETCH_SIZE gpurun_out/pmc_frames_WRITE_SIZE "gcm_frames_kernel<false>" $((64 * 41943040 + 64 * (41943040 + 28 * 640))) --what "gcm_frames_kernel<encrypt>, bench.py --config frames --objects 64; algorithmic = plaintext read + frames written" --out gpurun_out/pmc_gcm.json

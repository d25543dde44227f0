#!/bin/bash
# SHA-256 form A/B on the GPU box (replaces gpu_quad_check.sh):
#   scripts/gpu_sha_ab.sh <out-subdir> <ENV> <v1,v2[,...]> [extra env assignments...]
# Runs the SHA-256 GPU parity tests, then tools/sha_split_ab.py over config 3's
# verify launch (10 240 x 1 MiB) and three 10 MiB messages, alternating the
# values of ENV within one process.  Every step under its own time limit; the
# first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${1:?out subdir}"
ENVV=${2:?env var}
VALS=${3:?values}
shift 3
for kv in "$@"; do export "$kv"; done
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "sha256" -x -v --timeout 120 --timeout-method thread \
  > "$O/pytest_sha.log" 2>&1 || { tail -40 "$O/pytest_sha.log"; exit 1; }
tail -1 "$O/pytest_sha.log"
timeout -k 10 300 python tools/sha_split_ab.py --env "$ENVV" --values "$VALS" --messages 10240 \
  > "$O/ab_cfg3.jsonl" 2>&1 || { tail -20 "$O/ab_cfg3.jsonl"; exit 1; }
cat "$O/ab_cfg3.jsonl"
timeout -k 10 300 python tools/sha_split_ab.py --env "$ENVV" --values "$VALS" --messages 3 --size 10485760 \
  --rounds 2 --reps 2 > "$O/ab_10m.jsonl" 2>&1 || { tail -20 "$O/ab_10m.jsonl"; exit 1; }
cat "$O/ab_10m.jsonl"

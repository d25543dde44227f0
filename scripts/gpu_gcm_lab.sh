#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${GCM_VARIANTS:-default noaes noghash g3 g3_noghash}; do
  timeout -k 10 120 tools/gcm_lab_$v 64 $v >> gpurun_out/gcm_lab.jsonl 2>&1 || { cat gpurun_out/gcm_lab.jsonl; exit 1; }
done
cat gpurun_out/gcm_lab.jsonl

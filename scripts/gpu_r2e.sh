#!/bin/bash
# SHA stream-form debugging: the lab's check cases (digests vs split form,
# work words), then the stream GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r2e; mkdir -p $O
echo "== lab check"; timeout -k 10 120 tools/sha_stream_lab check > $O/lab_check.jsonl 2>&1; rc=$?; cat $O/lab_check.jsonl; echo "rc=$rc"
[ $rc -eq 0 ] || exit 1
echo "== lab big"; timeout -k 10 300 tools/sha_stream_lab big > $O/lab_big.jsonl 2>&1 || { cat $O/lab_big.jsonl; exit 1; }
cat $O/lab_big.jsonl

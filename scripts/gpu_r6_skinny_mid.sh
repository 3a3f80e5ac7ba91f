#!/bin/bash
# The skinny kernel at mid-size steps (256-1024 rows) for o / down vs the
# 256x256 tiles and hipBLASLt, plus its fp32 checks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm.py -x -q --timeout 120 --timeout-method thread -m gpu -k "skinny" > gpurun_out/sk_mid_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sk_mid_tests.log; [ $rc -eq 0 ] || exit $rc
SK_GEMMS=${SK_GEMMS:-o,down,qkv} SK_MS=${SK_MS:-256,300,384,512,640,768,1024} timeout -k 10 240 python -u bench/skinny_chunked.py > gpurun_out/sk_mid.jsonl 2>&1 || exit 1
cat gpurun_out/sk_mid.jsonl

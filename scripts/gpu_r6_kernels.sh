#!/bin/bash
# Kernel microbenchmarks of round 6: the skinny GEMM on a CU partition vs the
# chip (bench/skinny_partition.py) and the residual GEMM at the row counts
# hipBLASLt still serves (bench/resid_small_m.py).  Each step has its own
# time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 240 python -u bench/skinny_partition.py ${SKINNY_ARGS:-} 2>&1 | tee gpurun_out/r6_skinny_partition.jsonl || exit 1
timeout -k 10 240 python -u bench/resid_small_m.py 2>&1 | tee gpurun_out/r6_resid_small_m.jsonl || exit 1

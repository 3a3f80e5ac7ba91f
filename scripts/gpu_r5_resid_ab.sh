#!/bin/bash
# o / down residual GEMM: the LDS-staged residual epilogue (GM_EPI_RESID_LDS)
# against the register one and hipBLASLt beta = 1 -- fp32 numerics first,
# then interleaved timing rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm.py -q -x -k residual --timeout 120 --timeout-method thread \
  > gpurun_out/r5_resid_tests.log 2>&1 || { echo "resid tests failed"; tail -30 gpurun_out/r5_resid_tests.log; exit 1; }
tail -2 gpurun_out/r5_resid_tests.log
timeout -k 10 300 python bench/gemm_fused.py --resid --rounds 9 --iters 10 > gpurun_out/r5_resid_ab.jsonl 2> gpurun_out/r5_resid_ab.err \
  || { echo "resid bench failed"; tail -10 gpurun_out/r5_resid_ab.err; exit 1; }
grep '"bench": "resid"' gpurun_out/r5_resid_ab.jsonl

#!/bin/bash
# Round 5: the RMSNorm row scales from the residual GEMM's epilogue
# (gemm_residual_rms) instead of a separate row_rms pass.  GEMM numerics
# tests, then the serving A/B (default vs --no-fused-rms), alternating on one
# box, 100-step windows.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r5_fused_rms
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm.py -m gpu \
  > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
BENCH_T=300 bash scripts/gpu_bench_ab.sh "--steps 100 --warmup 5 --gateway-only-s 0 --slo-climb 0.5" \
  "--fused-rms" - "--fused-rms" - || exit $?
cp gpurun_out/bench_ab.jsonl $D/serving_ab.jsonl

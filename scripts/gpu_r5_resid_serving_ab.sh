#!/bin/bash
# Serving A/B of the o / down projections: hipBLASLt
# beta = 1 (--no-fused-resid) vs the hand-written residual GEMM with the
# epilogue variant RESID_EPI (the default since round 5 with lds),
# alternating on one box, 100-step windows.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
E=${RESID_EPI:-lds}
BENCH_T=300 bash scripts/gpu_bench_ab.sh "--steps 100 --warmup 5 --gateway-only-s 0 --slo-climb 0.5" \
  "--no-fused-resid" "--resid-epi $E" "--no-fused-resid" "--resid-epi $E" || exit $?
cp gpurun_out/bench_ab.jsonl gpurun_out/r5_resid_serving_ab_$E.jsonl

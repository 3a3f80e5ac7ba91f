#!/bin/bash
# PMC counter passes over the preprocess chain (text_analyze, embed_pool's
# MFMA embedding GEMM, classify_head, copies) at 4096 messages: one counter
# group per run, --kernel-trace --stats only, each pass bounded.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_text
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --stats -d gpurun_out/pmc_text/$name -o run \
    --output-format csv -- python3 bench/kernel_bench.py --only text --reps 20 \
    > gpurun_out/pmc_text/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES &&
pass mfma SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES &&
pass mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum

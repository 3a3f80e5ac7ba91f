#!/bin/bash
# PMC passes over the attention kernels at the serving step's shape
# (bench/kernel_bench.py --only attention: 768 decode tokens + 256 prefill
# chunks of 4-32, 32 / 64-key segment blocks, the long-context dialog case),
# one rocprofv3 run per counter group.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r5_attn_pmc
mkdir -p $D
A=(--only attention --reps 20)
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --stats -d $D/$name -o run --output-format csv \
    -- python3 bench/kernel_bench.py "${A[@]}" > $D/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
pass attn_mfma SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
pass attn_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES || exit 1
pass attn_fetch FETCH_SIZE || exit 1
pass attn_write WRITE_SIZE || exit 1

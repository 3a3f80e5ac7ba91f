#!/bin/bash
# GEMM energy diagnostic (bench/gemm_energy_diag.hip): wall-time A/B of the
# production kernel vs builds without LDS fragment reads / staging DMA, then
# one PMC pass for the shader clock (GRBM_GUI_ACTIVE / 8 / wall) and MFMA busy.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 bench/gemm_energy_diag 4096 28672 4096 9 > gpurun_out/energy_diag.jsonl 2>&1 || exit $?
timeout -k 10 120 bench/gemm_energy_diag 4096 4096 14336 9 >> gpurun_out/energy_diag.jsonl 2>&1 || exit $?
cat gpurun_out/energy_diag.jsonl
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
  --kernel-trace -d gpurun_out/pmc_energy -o pmc -- bench/gemm_energy_diag 4096 28672 4096 2 0 > gpurun_out/pmc_energy.log 2>&1
echo "pmc rc=$?"

#!/bin/bash
# PMC passes over the hand-written GEMM (bench/gemm_pmc.py), one rocprofv3 run per counter set.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gemm
set -e
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_gemm/p1 -o p1 --output-format csv -- python3 bench/gemm_pmc.py > gpurun_out/pmc_gemm/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_COUNT TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_gemm/p2 -o p2 --output-format csv -- python3 bench/gemm_pmc.py > gpurun_out/pmc_gemm/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_gemm/p3 -o p3 --output-format csv -- python3 bench/gemm_pmc.py > gpurun_out/pmc_gemm/p3.log 2>&1
find gpurun_out/pmc_gemm -name "*counter_collection*"

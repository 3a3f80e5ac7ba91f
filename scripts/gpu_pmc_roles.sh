#!/bin/bash
# PMC passes over the serving GEMM roles (bench/gemm_pmc_roles.py), one rocprofv3 run per counter set.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/pmc_roles
mkdir -p $D
set -e
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $D/p1 -o p1 --output-format csv -- python3 bench/gemm_pmc_roles.py > $D/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_COUNT TCC_HIT_sum TCC_MISS_sum -d $D/p2 -o p2 --output-format csv -- python3 bench/gemm_pmc_roles.py > $D/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 bench/gemm_pmc_roles.py > $D/kt.log 2>&1
find $D -name "*.csv" | head -20

#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 ${PROF_T:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 6} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc

#!/bin/bash
# rocprofv3 kernel trace of bench/micro_stress.py (the partition mode by
# default): per-kernel time of the serving steps and of the micro-forwards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/r6_prof_micro; mkdir -p gpurun_out/r6_prof_micro
timeout -k 10 ${PROF_T:-300} rocprofv3 --kernel-trace --stats -d gpurun_out/r6_prof_micro -o run --output-format csv \
  -- python3 bench/micro_stress.py --seconds ${SECONDS_RUN:-12} --report-s 3 ${STRESS_ARGS:---stream partition --micro-cus 32 --budget 3584 --slots 1344} \
  > gpurun_out/r6_prof_micro.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -4 gpurun_out/r6_prof_micro.log
find gpurun_out/r6_prof_micro -name "*.csv" | head
exit $rc

#!/bin/bash
# rocprofv3 kernel trace of bench/micro_stress.py (the partition mode by
# default): per-kernel time of the serving steps and of the micro-forwards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r6_prof_${TAG:-micro}
rm -rf $D; mkdir -p $D
timeout -k 10 ${PROF_T:-300} rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv \
  -- python3 bench/micro_stress.py --seconds ${SECONDS_RUN:-12} --report-s 3 ${STRESS_ARGS:---stream partition --micro-cus 32 --budget 3584 --slots 1344} \
  > $D.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v "^    @" $D.log | tail -4
[ $rc -eq 0 ] || exit $rc
# summaries on the box: the raw trace is too large to copy back
python scripts/trace_streams.py $D/run_kernel_trace.csv --top 6 > $D.streams.json
python scripts/timeline_excerpt.py $D/run_kernel_trace.csv --at 0.55 --ms ${EXCERPT_MS:-150} > $D.timeline.txt
python scripts/prof_summary.py $D/run > $D.md
rm -f $D/run_kernel_trace.csv
exit 0

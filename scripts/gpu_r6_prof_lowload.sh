#!/bin/bash
# rocprofv3 kernel trace of the 1-GPU bench at 30 % load (the library-free
# path's weak spot): per-kernel time of ~165-token steps.  Summaries are
# written on the box; the raw trace is deleted (too large to copy back).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r6_prof_${TAG:-lowload}
rm -rf $D; mkdir -p $D
timeout -k 10 ${PROF_T:-400} rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv \
  -- python3 bench.py --steps 60 --warmup 10 --util 0.3 --slo-climb= --slo-backoff= ${BENCH_ARGS:-} \
  > $D.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v "^    @" $D.log | tail -2 | cut -c1-600
[ $rc -eq 0 ] || exit $rc
python scripts/timeline_excerpt.py $D/run_kernel_trace.csv --at 0.55 --ms ${EXCERPT_MS:-40} > $D.timeline.txt
python scripts/prof_summary.py $D/run > $D.md
rm -f $D/run_kernel_trace.csv
exit 0

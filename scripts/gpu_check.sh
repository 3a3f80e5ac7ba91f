#!/bin/bash
# GPU validation sequence for gpurun: stop at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 ${PYTEST_T:-500} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_T:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
  exit $rc
fi

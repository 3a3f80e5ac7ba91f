#!/bin/bash
# QPS sweep on one MI355X (BASELINE config 3's "synthetic Poisson QPS sweep"):
# bench.py at a list of offered loads (fractions of the calibrated capacity),
# one JSON line per point into gpurun_out/qps_sweep.jsonl.  Each point is its
# own process (fresh calibration), bounded by its own timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/qps_sweep.jsonl
for u in ${UTILS:-0.5 0.7 0.8 0.9 0.95 1.0 1.05}; do
  timeout -k 10 ${PT_T:-240} python bench.py --steps ${STEPS:-60} --warmup 5 --util $u --gateway-only-s 0 \
    > gpurun_out/qps_$u.log 2>&1 || { echo "point $u failed rc=$?"; exit 1; }
  tail -1 gpurun_out/qps_$u.log >> gpurun_out/qps_sweep.jsonl
  echo "util $u done"
done

#!/bin/bash
# The 8-rank simulated-GPU rehearsals of round 4, re-run on a GPU box's CPU
# share (16 cores) instead of the 8-core build container, to separate CPU
# contention from design cost: bench.py --cpu-dry-run
# --sim-gpu at 8 ranks in both ingress modes, then the HTTP front door with 8
# `cli serve` ranks at 33k and 43k req/s.  Nothing here touches the GPU.
# Output: gpurun_out/box_sim_breakdown.jsonl, gpurun_out/box_http_8ranks.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "cpus in affinity: $(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
LOG=gpurun_out/box_sim_bench.log OUT=gpurun_out/box_sim_breakdown.jsonl WORLDS="${WORLDS:-8}" timeout -k 10 900 bash scripts/sim_breakdown.sh || exit $?
: > gpurun_out/box_http_8ranks.jsonl
for RATE in ${RATES:-33000 43000}; do
  timeout -k 10 240 python bench/http_load.py --spawn multirank --ranks 8 --sim-gpu 1,0.97,1.03 --bench-config \
    --client native --procs 2 --conns 16 --threads 2 --rate "$RATE" --duration 10 --warmup 3 --workload \
    --admin-churn 2 --server-log "gpurun_out/box_http_serve_$RATE.log" >> gpurun_out/box_http_8ranks.jsonl || exit $?
  tail -c 600 gpurun_out/box_http_8ranks.jsonl; echo
done

#!/bin/bash
# Fair vs greedy draining of the one shared front-door ring at 8 ranks, on a
# GPU box's 16-core CPU share (nothing touches the GPU): bench.py's rank0
# ingress sim with --door-share greedy / fair, then `cli serve` 8 ranks over
# HTTP (whose ring threads now take a 1/world fair share per pop) at 33k and
# 43k req/s.  Output under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for SH in ${SHARES:-greedy fair}; do
  LOG=gpurun_out/box_share_$SH.log OUT=gpurun_out/box_share_$SH.jsonl WORLDS=8 INGRESS=rank0 PINS=none \
    EXTRA="--door-share $SH" timeout -k 10 400 bash scripts/sim_breakdown.sh || exit $?
done
: > gpurun_out/box_http_8ranks_fair.jsonl
for RATE in ${RATES:-33000 43000}; do
  timeout -k 10 240 python bench/http_load.py --spawn multirank --ranks 8 --sim-gpu 1,0.97,1.03 --bench-config \
    --client native --procs 2 --conns 16 --threads 2 --rate "$RATE" --duration 10 --warmup 3 --workload \
    --admin-churn 2 --server-log "gpurun_out/box_http_fair_$RATE.log" >> gpurun_out/box_http_8ranks_fair.jsonl || exit $?
  python - <<'PY'
import json
d = json.loads(open("gpurun_out/box_http_8ranks_fair.jsonl").read().splitlines()[-1])
print(d["offered_rps"], d["accepted"], "ack p99", d["p99_ms"], "by rank", d["accepted_by_rank"],
      "p99 by tier", d["dispatcher"]["latency"]["p99_by_tier_ms"])
PY
done

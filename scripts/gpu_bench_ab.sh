#!/bin/bash
# A/B of bench.py variants on one MI355X, each run bounded; one JSON line per
# variant in gpurun_out/bench_ab.jsonl.  Usage:
#   bash scripts/gpu_bench_ab.sh "<common args>" "<variant args 1>" "<variant args 2>" ...
# (a variant "-" means no extra args)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
common=$1; shift
: > gpurun_out/bench_ab.jsonl
i=0
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  i=$((i + 1))
  timeout -k 10 ${BENCH_T:-300} python bench.py $common $v > gpurun_out/bench_ab_$i.log 2>&1
  rc=$?
  echo "variant $i ($v) rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_ab_$i.log; exit $rc; }
  python - "$v" gpurun_out/bench_ab_$i.log >> gpurun_out/bench_ab.jsonl <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps({"variant": sys.argv[1] or "default", "value": d["value"],
                  "calibrated": d["calibrated_capacity_per_gpu"], "backend_tokens_per_s": d["backend_tokens_per_s"],
                  "tick_ms_saturated": d["host_ms_per_tick_saturated"]["tick_ms"],
                  "gpu_step_ms": d["lockstep"]["gpu_step_ms_mean_by_rank"][0],
                  "p99_ms": d["p99_ms"], "p99_realtime_ms": d["p99_by_tier_ms"][0], "p99_e2e_ms": d["p99_e2e_ms"],
                  "targets_met": d["p99_target_met"] and d["p99_e2e_target_met"], "warm_shapes": d["warm_shapes"]}))
PY
  tail -1 gpurun_out/bench_ab.jsonl
done

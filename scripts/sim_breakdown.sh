#!/bin/bash
# Multi-rank latency attribution on the CPU: the 8-rank
# bench in simulated-GPU mode (SimEngine at the serving config, speeds
# 1 / 0.97 / 1.03 cycled over ranks) at 2, 4 and 8 ranks, per-rank and rank-0
# front-door ingress, with and without one core per rank.  One JSON line per
# run (bench.py's line + the run's knobs) into $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-profiles/r4_sim_breakdown.jsonl}
: > "$OUT"
for W in ${WORLDS:-2 4 8}; do
  for ING in ${INGRESS:-per-rank rank0}; do
    for PIN in ${PINS:-"" "--pin-cpu"}; do            # PINS=none: unpinned only
      [ "$PIN" = none ] && PIN=""
      timeout -k 10 900 python bench.py --gpus "$W" --cpu-dry-run --sim-gpu 1,0.97,1.03 --steps 100 --warmup 10 \
        --gateway-only-s 0 --ingress "$ING" $PIN $EXTRA --json-out /tmp/sim_breakdown.json > "${LOG:-/tmp/sim_breakdown.log}" 2>&1 || exit $?
      python - "$W" "$ING" "${PIN:-none}" "$OUT" "${EXTRA:-}" <<'PY'
import json, sys
d = json.load(open("/tmp/sim_breakdown.json"))
d["run"] = {"world": int(sys.argv[1]), "ingress": sys.argv[2], "pin": sys.argv[3], "extra": sys.argv[5]}
open(sys.argv[4], "a").write(json.dumps(d) + "\n")
lb = d["latency_breakdown"]
print(sys.argv[1], sys.argv[2], sys.argv[3], d["value"], "rt", d["p99_by_tier_ms"][0], "all", d["p99_ms"],
      "tiers", d["p99_by_tier_ms"], "queue p99", lb["queue"]["p99_ms"][-1], "ingress p99", lb["ingress"]["p99_ms"][-1])
PY
    done
  done
done

#!/bin/bash
# Step token budget vs realtime end-to-end latency on one MI355X (VERDICT r4
# missing #2): the bench at several (token budget, slots) pairs -- the
# per-step cost a realtime request pays 4 times (prefill + 3 decode) plus the
# run-ahead wait -- to price a realtime step cap.  CONFIGS: "budget:slots:inflight".
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r5_budget_sweep.jsonl
: > $out
for C in ${CONFIGS:-4096:1536:2 2048:1024:2 1536:768:2 1024:512:2 1536:768:1}; do
  IFS=: read -r B S I <<< "$C"
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --token-budget $B --slots $S --inflight $I \
    --gateway-only-s 0 ${EXTRA:-} > gpurun_out/r5_budget_${B}_${S}_${I}.json 2> gpurun_out/r5_budget_${B}_${S}_${I}.err \
    || { echo "bench $C failed rc=$?"; tail -5 gpurun_out/r5_budget_${B}_${S}_${I}.err; exit 1; }
  python - gpurun_out/r5_budget_${B}_${S}_${I}.json $B $S $I >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"token_budget": int(sys.argv[2]), "slots": int(sys.argv[3]), "inflight": int(sys.argv[4]),
                  "value": d["value"], "capacity": d["calibrated_capacity_per_gpu"], "util": d["config"]["util"],
                  "ms_per_step": d["ms_per_step"], "backend_tokens_per_s": d["backend_tokens_per_s"],
                  "p99_by_tier_ms": d["p99_by_tier_ms"], "p99_e2e_by_tier_ms": d["p99_e2e_by_tier_ms"],
                  "attempts": d["slo_search"]["attempts"]}))
PY
  tail -1 $out
done

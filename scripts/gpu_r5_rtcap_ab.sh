#!/bin/bash
# Realtime step cap A/B on one MI355X (VERDICT r4 missing #2): the default
# bench (4096-token steps, 1536 slots) with backend.realtime_step_tokens off
# and at CAPS, same box, back to back.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r5_rtcap_ab.jsonl
: > $out
for C in ${CAPS:-0 1024 1536 0}; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --gateway-only-s 0 --realtime-step-tokens $C \
    > gpurun_out/r5_rtcap_$C.json 2> gpurun_out/r5_rtcap_$C.err || { echo "cap $C failed rc=$?"; tail -5 gpurun_out/r5_rtcap_$C.err; exit 1; }
  python - gpurun_out/r5_rtcap_$C.json $C >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"realtime_step_tokens": int(sys.argv[2]), "value": d["value"], "util": d["config"]["util"],
                  "capacity": d["calibrated_capacity_per_gpu"], "ms_per_step": d["ms_per_step"],
                  "backend_tokens_per_s": d["backend_tokens_per_s"], "realtime_p99_e2e_ms": d["realtime_p99_e2e_ms"],
                  "p99_by_tier_ms": d["p99_by_tier_ms"], "p99_e2e_by_tier_ms": d["p99_e2e_by_tier_ms"],
                  "attempts": d["slo_search"]["attempts"]}))
PY
  tail -1 $out | cut -c1-400
done

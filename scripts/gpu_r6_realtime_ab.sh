#!/bin/bash
# Realtime modes A/B on one MI355X (VERDICT r5 missing #1, next #2): the
# default bench with backend.realtime_mode off / micro (high-priority stream,
# same stream) / cap, same box, back to back, plus the micro-mode GPU test.
# VARIANTS: ';'-separated "tag:extra bench args".
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_realtime_micro.py} -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r6_rt_pytest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6_rt_pytest.log; exit 1; }
  tail -2 gpurun_out/r6_rt_pytest.log
fi
out=gpurun_out/${OUT:-r6_realtime_ab}.jsonl
: > $out
IFS=';' read -ra VS <<< "${VARIANTS:-off:--realtime-mode off;micro:--realtime-mode micro;cap1024:--realtime-step-tokens 1024;micro_same:--realtime-mode micro --micro-stream same}"
for V in "${VS[@]}"; do
  tag=${V%%:*}
  args=${V#*:}
  timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 --gateway-only-s 0 $args \
    > gpurun_out/r6_rt_$tag.json 2> gpurun_out/r6_rt_$tag.err || { echo "$tag failed rc=$?"; tail -8 gpurun_out/r6_rt_$tag.err; exit 1; }
  python - gpurun_out/r6_rt_$tag.json "$tag" "$args" >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"tag": sys.argv[2], "args": sys.argv[3], "value": d["value"], "util": d["config"]["util"],
                  "realtime_mode": d.get("realtime_mode"), "capacity": d["calibrated_capacity_per_gpu"],
                  "ms_per_step": d["ms_per_step"], "backend_tokens_per_s": d["backend_tokens_per_s"],
                  "mfma_peak_fraction": d.get("mfma_peak_fraction"), "micro_forwards": d.get("micro_forwards"),
                  "realtime_p99_e2e_ms": d["realtime_p99_e2e_ms"], "p99_by_tier_ms": d["p99_by_tier_ms"],
                  "p99_e2e_by_tier_ms": d["p99_e2e_by_tier_ms"], "request_shape": d.get("request_shape"),
                  "host_ms_per_tick": d.get("host_ms_per_tick"), "attempts": d["slo_search"]["attempts"]}))
PY
  tail -1 $out | cut -c1-600
done

#!/bin/bash
# GEMM routing tests, then 30 %-load benches (library-free, --library-gemm)
# and the default saturated bench, one JSON line each into one file.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r6_lowload_ab${SUFFIX:-}.jsonl; : > $O
timeout -k 10 400 python -u -m pytest tests/test_gemm.py tests/test_realtime_micro.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/lowload_tests.log 2>&1; rc=$?; tail -2 gpurun_out/lowload_tests.log; [ $rc -eq 0 ] || exit $rc
for args in "--util 0.3 --slo-climb= --slo-backoff=" "--util 0.3 --slo-climb= --slo-backoff= --library-gemm" ""; do
  timeout -k 10 400 python -u bench.py $args > gpurun_out/lowload_bench.log 2>&1 || { tail -5 gpurun_out/lowload_bench.log; exit 1; }
  python - "$args" <<'PY' >> $O
import json, sys
d = json.loads(open("gpurun_out/lowload_bench.log").read().strip().splitlines()[-1])
keep = ("value", "ms_per_step", "util", "capacity", "backend_tokens_per_s", "mfma_peak_fraction", "realtime_p99_e2e_ms", "p99_by_tier_ms")
print(json.dumps({"args": sys.argv[1], **{k: d.get(k) for k in keep}}))
PY
  tail -1 $O
done

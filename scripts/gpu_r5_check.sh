#!/bin/bash
# Round-5 GPU check on one MI355X: the GPU test suite, the driver's default
# bench command, then the HTTP sequence the round-4 stalls followed (1-rank
# `cli serve` monolith, then 2 ranks time-sharing the GPU, in one call), with
# the per-incarnation segment names and the fatal stall watchdog in place.
# Every GPU step has its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r5_pytest_gpu.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r5_pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/r5_pytest_gpu.log
fi
if [ -z "${SKIP_SMOKE:-}" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r5_smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 gpurun_out/r5_smoke.log; exit 1; }
  echo "smoke ok"; tail -2 gpurun_out/r5_smoke.log
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err \
    || { echo "bench failed rc=$?"; tail -20 gpurun_out/r5_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r5_bench.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['p99_by_tier_ms'], d['p99_e2e_by_tier_ms'], d['slo_search']['util_tried'])"
fi
i=0
[ -n "${SKIP_HTTP:-}" ] && exit 0
for V in ${VARIANTS:-1:5300:--bench-config 2:5000:--bench-config}; do
  IFS=: read -r RANKS RATE EXTRA <<< "$V"
  i=$((i + 1))
  tag=r5_http_${RANKS}ranks_1gpu_${RATE}${EXTRA:+_bc}_$i
  timeout -k 10 300 python bench/http_load.py --spawn multirank --ranks "$RANKS" --gpu $EXTRA --client native \
    --workload --procs 2 --conns 16 --threads 2 --rate "$RATE" --duration 15 --warmup 10 --admin-churn 2 \
    --server-log gpurun_out/$tag.log > gpurun_out/$tag.json 2> gpurun_out/$tag.err
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - gpurun_out/$tag.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["accepted"], d.get("accepted_by_rank"), d["dispatcher"]["dispatch"]["dispatched"],
      d["dispatcher"]["dispatch"]["completed"], d["dispatcher"]["latency"]["p99_by_tier_ms"])
PY
done

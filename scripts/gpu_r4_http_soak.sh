#!/bin/bash
# Longer HTTP soak of `cli serve` on one MI355X (final round-4 code): 2 ranks
# time-sharing the GPU behind the C++ front door, bench config, admin churn,
# DURATION seconds measured.  The stall watchdog dumps stacks into the log if
# the serve loop stops ticking.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${RANKS:-2}; RATE=${RATE:-4500}; D=${DURATION:-120}
timeout -k 10 $((D + 240)) python bench/http_load.py --spawn multirank --ranks $R --gpu --bench-config --slots ${SLOTS:-1536} --client native \
  --workload --procs 2 --conns 16 --threads 2 --rate $RATE --duration $D --warmup 10 --admin-churn 5 \
  --cancel-churn ${CANCEL:-0} --dialog-frac ${DIALOG:-0} --dialog-convs ${CONVS:-5000} \
  --timeout-frac ${TOFRAC:-0} --timeout-val ${TOVAL:-150ms} --fault-cycle ${FAULTS:-0} \
  --server-log gpurun_out/http_soak_${R}r.log > gpurun_out/${TAG:-r4}_http_soak_${R}ranks_${RATE}_${D}s${SUFFIX:-}.json 2> gpurun_out/http_soak.err
rc=$?; echo "soak rc=$rc"; echo "stalls: $(grep -c stalled gpurun_out/http_soak_${R}r.log)"
python - gpurun_out/${TAG:-r4}_http_soak_${R}ranks_${RATE}_${D}s${SUFFIX:-}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["accepted"], d.get("accepted_by_rank"), d["dispatcher"]["dispatch"]["completed"], d["p99_ms"],
      d["dispatcher"]["latency"]["p99_by_tier_ms"], d.get("admin_churn"), d.get("cancel_churn"), d.get("fault_cycle"))
PY
exit $rc

#!/bin/bash
# The driver's 1-GPU bench command three times back to back on one box:
# the run-to-run spread of the headline on a single chip (box-to-box spread
# is larger: profiles/r5_* across calls).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r5_bench_repeat.jsonl
for i in 1 2 3; do
  timeout -k 10 400 python bench.py > gpurun_out/r5_bench_repeat_$i.json 2> gpurun_out/r5_bench_repeat_$i.err \
    || { echo "bench $i failed rc=$?"; tail -20 gpurun_out/r5_bench_repeat_$i.err; exit 1; }
  grep '^{' gpurun_out/r5_bench_repeat_$i.json | tail -1 | python3 -c "
import json,sys;d=json.loads(sys.stdin.read())
print(json.dumps({'run':$i,'value':d['value'],'ms_per_step':d['ms_per_step'],'capacity':d['calibrated_capacity_per_gpu'],'util':d['slo_search']['value_util'],'p99_by_tier_ms':d['p99_by_tier_ms'],'realtime_p99_e2e_ms':d['realtime_p99_e2e_ms']}))" | tee -a gpurun_out/r5_bench_repeat.jsonl
done

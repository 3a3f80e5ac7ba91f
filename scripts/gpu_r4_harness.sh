#!/bin/bash
# Round 4: util A/B of the 1-GPU bench (the SLO search makes a missed
# operating point report 0, so the offered util is a choice of margin), then
# 2-rank one-GPU rehearsals of the overload and dialog benches (both ranks
# share the one MI355X on gloo; not scaling measurements).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/h
: > gpurun_out/h/util_ab.jsonl
for i in 1 2; do
  for U in 1.0 0.98; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --util $U --gateway-only-s 0 --json-out gpurun_out/h/u.json > gpurun_out/h/u.log 2>&1
    rc=$?; echo "bench util $U rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cat gpurun_out/h/u.json >> gpurun_out/h/util_ab.jsonl
  done
done
timeout -k 10 420 python bench/overload_bench.py --gpus 2 --seconds 8 --fault-every 60 --autoscale 1.5:5,0.1:5,1.5:5 \
  --scale-cooldown-s 1.0 --json-out gpurun_out/h/overload_2ranks.json > gpurun_out/h/overload.log 2>&1
rc=$?; echo "overload rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python bench/dialog_bench.py --gpus 2 --convs 256 --turns 6 --ingress rank0 \
  --json-out gpurun_out/h/dialog_2ranks_rank0.json > gpurun_out/h/dialog.log 2>&1
rc=$?; echo "dialog rc=$rc"; exit $rc

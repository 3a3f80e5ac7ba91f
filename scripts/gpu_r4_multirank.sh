#!/bin/bash
# Round-4 GPU check: GPU tests, the driver's 1-GPU bench, then the 2-rank
# one-GPU rehearsal at the DEFAULT serving budgets in both ingress modes
# (two ranks share the one MI355X on gloo; not a scaling measurement).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/r4_bench_1gpu.json > gpurun_out/r4_bench_1gpu.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
for ING in per-rank rank0; do
  timeout -k 10 420 python bench.py --gpus 2 --steps 40 --warmup 10 --gateway-only-s 0 --ingress $ING \
    --json-out gpurun_out/r4_2ranks_1gpu_$ING.json > gpurun_out/r4_2ranks_1gpu_$ING.log 2>&1
  rc=$?; echo "2-rank $ING rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

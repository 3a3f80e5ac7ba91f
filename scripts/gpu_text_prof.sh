#!/bin/bash
# Per-kernel times of the preprocess chain at several batch sizes
# (rocprofv3 --kernel-trace --stats only), plus the un-profiled pipeline times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
tag=${1:-base}
mkdir -p gpurun_out/text_$tag
for b in 64 256 512 4096; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/text_$tag/b$b -o run --output-format csv \
    -- python3 bench/kernel_bench.py --only text --reps 100 --text-batches $b > gpurun_out/text_$tag/b$b.log 2>&1 || exit $?
done
timeout -k 10 120 python3 bench/kernel_bench.py --only text --reps 100 --text-batches 64,256,512,4096 \
  > gpurun_out/text_$tag/plain.log 2>&1

#!/bin/bash
# Lock-step vs extra local steps on one MI355X (2 ranks time-share the GPU;
# rank 1 takes half-size steps, so it is the "faster" rank), the 1-GPU
# headline (world 1 is unaffected by the change), and the GPU suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_tests.txt
for x in "" "--no-extra-steps"; do
  tag=${x:-extra}
  timeout -k 10 300 python bench.py --gpus 2 --slots 768 --steps 60 --warmup 5 --gateway-only-s 0 \
      --token-budget-by-rank 1:2048 $x > gpurun_out/xs_$tag.json 2> gpurun_out/xs_$tag.err || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err || exit 1
echo done

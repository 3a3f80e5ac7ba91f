#!/bin/bash
# A/B of the attention segment kernel's K/V staging (round 5): all loads of
# a key block in flight before the LDS stores (new, _lib) vs the round-4
# per-item predicated loads (ab_lib/old, built from the previous commit).
# Numerics first, then alternating kernel_bench attention runs.  ab_lib/old is
# built on the CPU beforehand: check out the old llama_kernels.h, run
# `python -m llm_message_queue_amd._build --only _hipops --force`, copy every
# _lib/*.so to ab_lib/old, restore the new header and build again.  Result
# (round 5): the new form was 18 % slower and was reverted
# (profiles/r5_attn_ab.jsonl).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r5_attn_ab
mkdir -p $D
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "attention or tiny_model" > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for i in 1 2 3; do
  for V in old new; do
    LIB=""; [ $V = old ] && LIB="--lib-dir ab_lib/old"
    timeout -k 5 120 python3 bench/kernel_bench.py --only attention --reps 100 $LIB > $D/${V}_$i.log 2>&1 || { echo "$V $i failed"; tail -5 $D/${V}_$i.log; exit 1; }
    echo "$V $i $(grep '^{"kernel' $D/${V}_$i.log | python3 -c "import sys,json;print(' '.join(f\"{d['kernel']}={d['ms']}\" for d in map(json.loads,sys.stdin)))")"
  done
done

#!/bin/bash
# A/B of the qkv GEMM's split-K tail block mapping (round 5): XCD-contiguous
# remap of the tail blocks (new, _lib) vs the round-4 one-half-of-every-4th-
# tile mapping (ab_lib/old, built on the CPU from the previous commit's
# gemm_kernels.h).  Numerics first, then alternating bench/qkv_sweep.py runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r5_qkv_tail_ab
mkdir -p $D
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm.py -m gpu \
  > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for i in 1 2 3; do
  for V in old new; do
    LIB=""; [ $V = old ] && LIB="--lib-dir ab_lib/old"
    timeout -k 5 120 python3 bench/qkv_sweep.py --tokens 4041,4096,2048 --iters 50 $LIB > $D/${V}_$i.log 2>&1 \
      || { echo "$V $i failed"; tail -5 $D/${V}_$i.log; exit 1; }
    echo "$V $i $(grep '^{' $D/${V}_$i.log | python3 -c "import sys,json;print(' '.join(f\"T{d['T']}:split={d['qkv_rope_split_ms']},nosplit={d['qkv_rope_nosplit_ms']}\" for d in map(json.loads,sys.stdin)))")"
  done
done

#!/bin/bash
# Round-5 kernel rework check: summarise_project (K-split, flat mean pass),
# salient_topk (wave-level top-K), kv_move (chunked, 8 loads in flight,
# non-temporal): numerics tests, then standalone timing, one PMC pass of
# each summarise configuration (LDS + MFMA counters) and kv_move beyond the
# Infinity Cache.  Every GPU step bounded; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r5_k2
mkdir -p $D
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_migration.py \
  > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for N in ${SIZES:-64 256 4096}; do
  A=(--only text --text-batches $N --reps 20)
  timeout -k 5 120 python3 bench/kernel_bench.py "${A[@]}" > $D/time_text_$N.log 2>&1 || exit 1
  grep '^{"kernel' $D/time_text_$N.log
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d $D/text${N}_write -o run --output-format csv \
    -- python3 bench/kernel_bench.py "${A[@]}" > $D/text${N}_write.log 2>&1 || { echo "pmc write text $N failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-trace --stats -d $D/text${N}_mfma -o run --output-format csv \
    -- python3 bench/kernel_bench.py "${A[@]}" > $D/text${N}_mfma.log 2>&1 || { echo "pmc mfma text $N failed"; exit 1; }
done
for C in ${CONVS:-16 64 256}; do
  A=(--only summarise --summ-convs $C --reps 20)
  timeout -k 5 120 python3 bench/kernel_bench.py "${A[@]}" > $D/time_summ_$C.log 2>&1 || exit 1
  grep '^{"kernel' $D/time_summ_$C.log
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES \
    --kernel-trace --stats -d $D/summ${C}_lds -o run --output-format csv \
    -- python3 bench/kernel_bench.py "${A[@]}" > $D/summ${C}_lds.log 2>&1 || { echo "pmc lds $C failed"; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d $D/summ${C}_write -o run --output-format csv \
    -- python3 bench/kernel_bench.py "${A[@]}" > $D/summ${C}_write.log 2>&1 || { echo "pmc write $C failed"; exit 1; }
done
KV_VARIANTS=${KV_VARIANTS:-0,1,2} timeout -k 10 240 python3 bench/kv_move_bench.py > $D/kv_move.json 2> $D/kv_move.err \
  || { echo "kv_move failed"; tail -5 $D/kv_move.err; exit 1; }
grep '^{' $D/kv_move.json | python3 -c "import json,sys;d=json.loads(sys.stdin.readline());print(d['kv_move']);print(d.get('beyond_cache'))"

#!/bin/bash
# Round-5 kernel evidence for the north-star preprocess / summarise kernels
#  at serving batch sizes, standalone: per batch size one
# timing run, then one rocprofv3 pass per counter group (--kernel-trace
# --stats only; each pass bounded).  Then kv_move beyond the Infinity Cache.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
D=gpurun_out/r5_kpmc
mkdir -p $D
pass() {   # name, bench args..., --, counters...
  local name=$1; shift
  local args=()
  while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --stats -d $D/$name -o run --output-format csv \
    -- python3 bench/kernel_bench.py "${args[@]}" > $D/$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"; return $rc
}
for N in ${SIZES:-64 256 4096}; do
  A=(--only text --text-batches $N --reps 20)
  timeout -k 5 120 python3 bench/kernel_bench.py "${A[@]}" > $D/time_text_$N.log 2>&1 || exit 1
  pass text${N}_mfma "${A[@]}" -- SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
  pass text${N}_lds "${A[@]}" -- SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES || exit 1
  pass text${N}_fetch "${A[@]}" -- FETCH_SIZE || exit 1
  pass text${N}_write "${A[@]}" -- WRITE_SIZE || exit 1
done
for C in ${CONVS:-16 64 256}; do
  A=(--only summarise --summ-convs $C --reps 20)
  timeout -k 5 120 python3 bench/kernel_bench.py "${A[@]}" > $D/time_summ_$C.log 2>&1 || exit 1
  pass summ${C}_mfma "${A[@]}" -- SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 1
  pass summ${C}_lds "${A[@]}" -- SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES || exit 1
  pass summ${C}_fetch "${A[@]}" -- FETCH_SIZE || exit 1
  pass summ${C}_write "${A[@]}" -- WRITE_SIZE || exit 1
done
timeout -k 10 180 python3 bench/kv_move_bench.py > $D/kv_move.json 2> $D/kv_move.err || { echo "kv_move failed"; tail -5 $D/kv_move.err; exit 1; }
grep '^{' $D/kv_move.json | python3 -c "import json,sys;d=json.loads(sys.stdin.readline());print(d.get('beyond_cache'))"

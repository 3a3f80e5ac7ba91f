#!/bin/bash
# KV-migration data plane on one MI355X: kv_move pack/unpack bandwidth and a
# world-1 RCCL self-p2p sweep (bench/kv_move_bench.py, plain and under
# rocprofv3 --kernel-trace --stats), then the 2-rank migrate / replay
# rehearsal with the migrator's host time per migration tick.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kv
timeout -k 10 240 python bench/kv_move_bench.py > gpurun_out/kv/kv_move.json 2> gpurun_out/kv/kv_move.err
rc=$?; echo "kv_move rc=$rc"; tail -c 1500 gpurun_out/kv/kv_move.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/kv/prof -o kv --output-format csv -- python3 bench/kv_move_bench.py > gpurun_out/kv/prof.log 2>&1
rc=$?; echo "kv prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for MODE in migrate replay; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 200)) bench/migrate_bench.py --mode $MODE --convs 256 --turns 6 \
    > gpurun_out/kv/migrate_$MODE.log 2>&1
  rc=$?; echo "migrate $MODE rc=$rc"; grep "^{" gpurun_out/kv/migrate_$MODE.log | tail -c 1200; [ $rc -eq 0 ] || exit $rc
done

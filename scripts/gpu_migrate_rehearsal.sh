#!/bin/bash
# KV migration vs replay vs pinned on 1x MI355X (2 ranks share the GPU: gloo
# data plane, a functional rehearsal -- not an xGMI measurement).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/r3_migrate_bench.jsonl
: > $out
for mode in migrate replay pinned; do
  timeout -k 10 ${MB_T:-240} python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) bench/migrate_bench.py --mode $mode \
    ${MB_ARGS:-} > gpurun_out/migrate_$mode.log 2>&1 || { echo "migrate_bench $mode failed"; tail -20 gpurun_out/migrate_$mode.log; exit 1; }
  grep '^{' gpurun_out/migrate_$mode.log >> $out
done
cat $out

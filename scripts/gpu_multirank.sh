#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box: NPROC ranks share the one
# MI355X (devices wrap round, every group on gloo -- RCCL needs one device per
# rank).  Exercises the per-tick all_gather / all_to_all dispatch path, the
# global drain condition and the rank-0 report with real HIP backends.  Not a
# scaling measurement (the ranks split one GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
NPROC=${NPROC:-2}
timeout -k 10 ${MR_T:-420} python -m torch.distributed.run --nnodes=1 --nproc-per-node $NPROC \
  --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus $NPROC \
  ${MR_ARGS:---steps 40 --warmup 10 --slots 384 --gateway-only-s 1} > gpurun_out/multirank.log 2>&1
rc=$?; echo "multirank rc=$rc"; tail -4 gpurun_out/multirank.log
exit $rc

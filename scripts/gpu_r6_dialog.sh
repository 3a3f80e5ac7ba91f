#!/bin/bash
# Round 6: the long-dialog bench with real dialog context (prompt ids plus
# the generated ids read back per step; cross-rank replays carry the real
# history in K_HIST rows).  One rank on the MI355X (residency vs replay),
# then 2 ranks time-sharing it with every turn entering at rank 0, so half
# the turns are served remotely from replayed history (not a scaling run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/dlg6
timeout -k 10 300 python bench/dialog_bench.py --json-out gpurun_out/dlg6/dialog_1gpu.json \
  > gpurun_out/dlg6/dialog_1gpu.log 2>&1
rc=$?; echo "dialog 1 rank rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/dlg6/dialog_1gpu.log; exit $rc; }
timeout -k 10 420 python bench/dialog_bench.py --gpus 2 --convs 256 --turns 6 --ingress rank0 \
  --json-out gpurun_out/dlg6/dialog_2ranks_rank0.json > gpurun_out/dlg6/dialog_2r.log 2>&1
rc=$?; echo "dialog 2 ranks rc=$rc"; [ $rc -eq 0 ] || tail -20 gpurun_out/dlg6/dialog_2r.log; exit $rc

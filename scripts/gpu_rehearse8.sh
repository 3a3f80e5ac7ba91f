#!/bin/bash
# One-GPU rehearsal of the driver's 8-GPU scaling command: `bench.py --gpus 8`
# WITHOUT a launcher (bench.py starts torch.distributed.run itself), 8 ranks
# wrapped onto the one MI355X (every group on gloo -- RCCL needs one device per
# rank), both ingress modes.  Not a scaling measurement: the ranks split one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${R8_ARGS:---steps 20 --warmup 5 --slots 128 --gateway-only-s 1}
timeout -k 10 ${R8_T:-420} python bench.py --gpus 8 $ARGS --ingress ${R8_INGRESS:-per-rank} \
  > gpurun_out/rehearse8_${R8_INGRESS:-per-rank}.log 2>&1
rc=$?; echo "rehearse8 ${R8_INGRESS:-per-rank} rc=$rc"; tail -c 1500 gpurun_out/rehearse8_${R8_INGRESS:-per-rank}.log
exit $rc

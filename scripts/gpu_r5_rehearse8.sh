#!/bin/bash
# The driver's 8-GPU command shape on the one-GPU box, round-5 code:
# torch.distributed.run --nproc-per-node 8 bench.py --gpus 8, the 8 ranks
# time-sharing the MI355X (gloo data plane: RCCL needs one device per rank),
# 128 slots per rank so 8 copies of the 8B model and their KV fit in 288 GB.
# A control-flow rehearsal (SLO search, job tokens, CPU binding, accounting),
# not a scaling measurement.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PORT=$((20000 + RANDOM % 20000))
timeout -k 10 ${R8_T:-600} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port $PORT bench.py --gpus 8 --steps 20 --warmup 5 --slots 128 --gateway-only-s 0 \
  > gpurun_out/r5_rehearse8.json 2> gpurun_out/r5_rehearse8.err
rc=$?; echo "rehearse8 rc=$rc"
[ $rc -eq 0 ] || { tail -30 gpurun_out/r5_rehearse8.err; exit $rc; }
python3 - gpurun_out/r5_rehearse8.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
cb = d["comm"].get("cpu_binding", {})
print(d["n_gpus"], d["value"], d["slo_search"]["util_tried"], d["requests_accounted"], d["comm"]["data_backend"],
      cb.get("mode"), [(r["numa_node"], r["ncpus"]) for r in cb.get("by_rank", [])])
PY

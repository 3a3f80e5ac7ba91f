#!/bin/bash
# The driver's multi-GPU command shape on the one-GPU box (N=2: self-launch
# under torch.distributed.run, two ranks time-sharing the card over gloo --
# a control-flow rehearsal, not a scaling measurement), round-5 code: GPU-
# local CPU binding, job tokens, bidirectional SLO search.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for ING in per-rank rank0; do
  timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --ingress $ING \
    > gpurun_out/r5_rehearse2_$ING.json 2> gpurun_out/r5_rehearse2_$ING.err \
    || { echo "rehearse2 $ING failed rc=$?"; tail -20 gpurun_out/r5_rehearse2_$ING.err; exit 1; }
  python3 - gpurun_out/r5_rehearse2_$ING.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
cb = d["comm"].get("cpu_binding", {})
print(d["n_gpus"], d["value"], d["slo_search"]["util_tried"], d["requests_accounted"],
      cb.get("mode"), cb.get("source"), [(r["numa_node"], r["ncpus"], r["threads_bound"]) for r in cb.get("by_rank", [])])
PY
done

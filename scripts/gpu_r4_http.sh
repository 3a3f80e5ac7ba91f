#!/bin/bash
# Round-4 HTTP evidence on one MI355X with the final code: `cli serve` behind
# its C++ front door with 1 rank (the monolith) and with 2 ranks time-sharing
# the GPU (ring threads drain the shared ring with the balanced share), the
# bench serving config, admin churn on.  VARIANTS: "ranks:rate:extra" items.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for V in ${VARIANTS:-1:5300:--bench-config 2:5000:--bench-config}; do
  IFS=: read -r RANKS RATE EXTRA <<< "$V"
  i=$((i + 1))
  tag=r4_http_${RANKS}ranks_1gpu_${RATE}${EXTRA:+_bc}${REPEAT_TAG:+_$i}
  timeout -k 10 300 python bench/http_load.py --spawn multirank --ranks "$RANKS" --gpu $EXTRA --client native \
    --workload --procs 2 --conns 16 --threads 2 --rate "$RATE" --duration 15 --warmup 10 --admin-churn 2 \
    --server-log gpurun_out/$tag.log > gpurun_out/$tag.json 2> gpurun_out/$tag.err
  rc=$?; echo "$tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - gpurun_out/$tag.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["accepted"], d.get("accepted_by_rank"), d["dispatcher"]["dispatch"], d["dispatcher"]["latency"]["count"],
      d["dispatcher"]["latency"]["p99_by_tier_ms"])
PY
done

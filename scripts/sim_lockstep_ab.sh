#!/bin/bash
# Lock-step vs extra local steps on simulated GPUs (CPU only): bench.py's
# multi-rank control flow with SimEngine backends at the given relative
# speeds.  Usage: scripts/sim_lockstep_ab.sh WORLD SPEEDS OUT.jsonl
set -euo pipefail
W=$1; SPEEDS=$2; OUT=$3
: > "$OUT"
for x in "" "--no-extra-steps"; do
  timeout 1200 python bench.py --gpus "$W" --cpu-dry-run --sim-gpu "$SPEEDS" --steps 100 --warmup 5 \
      --gateway-only-s 0 $x 2>/dev/null | grep '^{' >> "$OUT"
done

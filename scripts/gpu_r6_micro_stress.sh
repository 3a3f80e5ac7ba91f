#!/bin/bash
# Micro-forward streams under load (bench/micro_stress.py): optional GPU
# tests first, then VARIANTS in order, each under its own time limit; the
# first failure ends the call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r6_stress_pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 gpurun_out/r6_stress_pytest.log; exit 1; }
  tail -2 gpurun_out/r6_stress_pytest.log
fi
IFS=';' read -ra VS <<< "${VARIANTS:-same:--stream same;high_rocblas:--stream high --blas rocblas;high_lt:--stream high --blas lt}"
for V in "${VS[@]}"; do
  tag=${V%%:*}
  args=${V#*:}
  echo "== $tag ($args)"
  timeout -k 10 ${LIMIT:-200} python -u bench/micro_stress.py --seconds ${SECONDS_RUN:-40} $args \
    2> gpurun_out/r6_stress_$tag.err | tee gpurun_out/r6_stress_$tag.jsonl
  rc=${PIPESTATUS[0]}
  echo "$tag rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/r6_stress_$tag.err; exit $rc; }
done

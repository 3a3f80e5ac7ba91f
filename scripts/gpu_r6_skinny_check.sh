set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm.py -x -q --timeout 120 --timeout-method thread -m gpu -k "skinny or library_free or swiglu" > gpurun_out/sk_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench/skinny_chunked.py > gpurun_out/sk_chunked_new.jsonl 2>&1 || exit 1
cat gpurun_out/sk_chunked_new.jsonl

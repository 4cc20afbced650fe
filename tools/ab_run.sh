set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -v -k bucket_tables --timeout 120 --timeout-method thread > gpurun_out/check/bucket.log 2>&1 || { tail -40 gpurun_out/check/bucket.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/check/bucket.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -30 gpurun_out/check/tests.log; exit 1; }
tail -2 gpurun_out/check/tests.log

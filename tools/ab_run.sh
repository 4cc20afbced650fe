set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/check
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -30 gpurun_out/check/tests.log; exit 1; }
tail -2 gpurun_out/check/tests.log
bash tools/ab_variants.sh c4 "local_table" nobkt
OPT_ARGS=--adjoint bash tools/ab_variants.sh c3 "local_table" nobkt
mkdir -p gpurun_out/ab3; mv gpurun_out/ab/c3_* gpurun_out/ab3/
bash tools/ab_variants.sh c3 "local_table" nobkt

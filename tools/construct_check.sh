set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ct
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_construct.py > gpurun_out/ct/tests.log 2>&1 || { tail -40 gpurun_out/ct/tests.log; exit 1; }
tail -3 gpurun_out/ct/tests.log
for c in c2 c3 c4 c5; do
  timeout -k 10 120 python tools/operator_time.py --config $c --reps 9 >> gpurun_out/ct/times.jsonl
  SPHRT_CONSTRUCT=python timeout -k 10 120 python tools/operator_time.py --config $c --reps 9 >> gpurun_out/ct/times.jsonl
done
cut -c1-170 gpurun_out/ct/times.jsonl

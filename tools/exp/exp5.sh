set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/exp5/gpu_tests.log 2>&1 || { tail -30 gpurun_out/exp5/gpu_tests.log; exit 1; }
tail -2 gpurun_out/exp5/gpu_tests.log
for c in c5 c2; do timeout -k 10 200 python tools/cold_breakdown.py --config $c > gpurun_out/exp5/cold_$c.log 2>&1; tail -1 gpurun_out/exp5/cold_$c.log; done
rm -rf gpurun_out/exp5/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp5/prof -o c5 --output-format csv -- python tools/cold_breakdown.py --config c5 --reps 2 > gpurun_out/exp5/c5p.log 2>&1
for f in $(find gpurun_out/exp5/prof -name "*kernel_stats.csv"); do cut -c1-150 "$f" | head -8; done

set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp3
rm -rf gpurun_out/exp3/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp3/prof -o c5 --output-format csv -- python tools/cold_breakdown.py --config c5 --reps 2 > gpurun_out/exp3/c5.log 2>&1
for f in $(find gpurun_out/exp3/prof -name "*kernel_stats.csv"); do cut -c1-200 "$f" | head -20; done

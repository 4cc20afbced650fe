set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp2
for c in c2 c5; do timeout -k 10 200 python tools/cold_breakdown.py --config $c > gpurun_out/exp2/cold_$c.log 2>&1; cat gpurun_out/exp2/cold_$c.log; done
timeout -k 10 120 python tools/host_overhead.py > gpurun_out/exp2/host.log 2>&1; cat gpurun_out/exp2/host.log

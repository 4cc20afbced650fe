set -e
export TMPDIR=/tmp
rocprofv3 --kernel-trace -d gpurun_out/gaps2 -o run --output-format csv -- python tools/operator_time.py --config c2 --reps 5 > /dev/null 2>&1
python tools/kernel_gaps.py gpurun_out/gaps2 8 | tail -32
timeout -k 10 120 python tools/prelude_time.py c2

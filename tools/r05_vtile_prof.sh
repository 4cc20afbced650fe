set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/vtprof; mkdir -p $O
for m in natural vtile:64,1,2; do
  n=$(echo $m | tr ':,' '__')
  SPHRT_RAY_ORDER=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- python tools/operator_time.py --config c3 --reps 3 > /dev/null 2>&1
done

#!/bin/bash
# A/B of the staged table build's row lookup (LDS row ids vs binary search, variant
# libsphrt_oldgather from the previous commit's apply.hip): rocprofv3 kernel stats of Operator
# construction (tools/operator_time.py) at C2 / C3 / C5, two interleaved rounds; then the
# table / staging tests on the new library.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/gather; mkdir -p $O
V=sph_raytracer_amd/lib/variants/libsphrt_oldgather.so
for i in 1 2; do
  for c in c3 c5 c2; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/new_${c}_$i -o run --output-format csv -- python tools/operator_time.py --config $c --reps 5 > $O/new_${c}_$i.json 2>/dev/null
    SPHRT_LIB=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/old_${c}_$i -o run --output-format csv -- python tools/operator_time.py --config $c --reps 5 > $O/old_${c}_$i.json 2>/dev/null
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_construct.py tests/test_gpu_fullsize.py tests/test_gpu_properties.py -k "native or c2_full or c5_full or c3_full or staged or onepass" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log

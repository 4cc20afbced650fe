#!/bin/bash
# Round 6: reference-mode trace — invalid=True with 4 waves per ray (tree) against one (variant
# w1), interleaved; the api-surface tests; rocprofv3 kernel stats of the C2 float32 and invalid
# Operator constructions.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_reference_suite.py -x -q --timeout 300 --timeout-method thread > $O/refmode_tests2.log 2>&1
tail -1 $O/refmode_tests2.log
for r in 1 2; do
  for v in tree w1; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/operator_time.py --config c2 --reps 7 --invalid 2>/dev/null | sed "s/^/{\"v\": \"$v\", \"x\": /; s/$/}/" >> $O/r06_refmode_inv_ab.jsonl
  done
done
cut -c1-200 $O/r06_refmode_inv_ab.jsonl
for m in f32 inv; do
  a="--ftype float32"; [ $m = inv ] && a="--invalid"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/op_ref_$m -o run --output-format csv -- python tools/operator_time.py --config c2 --reps 5 $a > $O/op_ref_$m.json 2> $O/op_ref_$m.err
  cp $(find $O/op_ref_$m -name "*kernel_stats.csv" | head -1) $O/r06_operator_c2_${m}_kernel_stats.csv
  head -6 $O/r06_operator_c2_${m}_kernel_stats.csv | cut -c1-150
done

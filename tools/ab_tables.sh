set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_properties.py -m gpu -x -v --timeout 200 --timeout-method thread -k "hash_tables or granule_tables or onepass_tables" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in radix hash radix hash; do  # A/B: full sort vs hash-deduplicated sort
  SPHRT_TABLE_SORT=$m timeout -k 10 200 python tools/operator_time.py --config c3 >> $O/op_c3.jsonl
  SPHRT_TABLE_SORT=$m timeout -k 10 200 python tools/operator_time.py --config c4 >> $O/op_c4.jsonl
done
cat $O/op_c3.jsonl $O/op_c4.jsonl
for m in radix hash; do
  SPHRT_TABLE_SORT=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o run --output-format csv -- python tools/operator_time.py --config c3 --reps 3 > /dev/null 2>&1
  f=$(find $O/prof_$m -name "*kernel_stats.csv"); cp $f $O/c3_${m}_kernel_stats.csv; grep -i "table\|compact" $f | cut -c1-160
done
for v in cu8 cb64k cu8b; do
  SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python tools/operator_time.py --config c3 --reps 3 > $O/op_$v.json 2>&1
  f=$(find $O/prof_$v -name "*kernel_stats.csv"); cp $f $O/c3_${v}_kernel_stats.csv; echo $v; grep -i "compact" $f | cut -c1-160
done

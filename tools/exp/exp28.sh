set -e
export TMPDIR=/tmp
for v in base m8; do
L=sph_raytracer_amd/lib/variants/libsphrt_$v.so; [ $v = base ] && L=sph_raytracer_amd/lib/libsphrt.so
for c in c3 c2; do
rm -rf gpurun_out/tb_${v}_$c
SPHRT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tb_${v}_$c -o tb --output-format csv -- python tools/trace_bench.py $c > gpurun_out/tb_${v}_$c.log 2>&1
done; done
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_m8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_properties.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1

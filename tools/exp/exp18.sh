set -e
export TMPDIR=/tmp
for v in a1 a2 a3 a4; do
rm -rf gpurun_out/abl_$v
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abl_$v -o s --output-format csv -- python tools/trace_bench.py c2 > gpurun_out/abl_$v.log 2>&1 || true
done

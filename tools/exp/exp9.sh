set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests9.log 2>&1 || { tail -40 gpurun_out/gpu_tests9.log; exit 1; }
tail -1 gpurun_out/gpu_tests9.log
for c in c2 c5 c3; do
echo "== $c product"; timeout -k 10 300 python tools/prof_forward.py --config $c --rounds 3 2>&1 | grep -v amdgpu | cut -c1-100
echo "== $c m7"; SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_m7.so timeout -k 10 300 python tools/prof_forward.py --config $c --rounds 3 2>&1 | grep "_f32" | cut -c1-100
echo "== $c m64_6"; SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_m64_6.so timeout -k 10 300 python tools/prof_forward.py --config $c --rounds 3 2>&1 | grep "_f64" | cut -c1-100
done

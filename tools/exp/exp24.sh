set -e
export TMPDIR=/tmp
for v in base lds64 lds80; do
L=sph_raytracer_amd/lib/variants/libsphrt_$v.so; [ $v = base ] && L=sph_raytracer_amd/lib/libsphrt.so
echo "== $v"; SPHRT_LIB=$L timeout -k 10 300 python tools/prof_forward.py --config c5 --rounds 3 2>&1 | grep -v amdgpu | grep -v atomic | cut -c1-100
done

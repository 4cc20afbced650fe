set -e
export TMPDIR=/tmp
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_stamps.so timeout -k 10 120 python tools/fwd_timeline.py c2 2>&1 | grep -v amdgpu | head -60

set -e
export TMPDIR=/tmp
for c in c2 c5; do SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so timeout -k 10 120 python tools/trace_phases.py $c 2>&1 | grep -v amdgpu; done

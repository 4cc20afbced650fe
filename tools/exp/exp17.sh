set -e
export TMPDIR=/tmp
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so timeout -k 10 120 python tools/trace_phases.py c2 > gpurun_out/tphase.log 2>&1 || echo "rc=$?"
grep -v amdgpu gpurun_out/tphase.log | tr -d '\n ' ; echo

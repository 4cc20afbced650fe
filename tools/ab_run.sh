set -e
export TMPDIR=/tmp
bash tools/abl_trace.sh c3 r04b
mkdir -p gpurun_out/stamps
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so timeout -k 10 180 python tools/trace_phases.py c3 > gpurun_out/stamps/c3.json 2> gpurun_out/stamps/c3.err
cat gpurun_out/stamps/c3.json

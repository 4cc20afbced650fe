set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/exp6/gpu_tests.log 2>&1 || { tail -30 gpurun_out/exp6/gpu_tests.log; exit 1; }
tail -1 gpurun_out/exp6/gpu_tests.log
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so timeout -k 10 120 python tools/exact_phases.py c5
timeout -k 10 200 python tools/cold_breakdown.py --config c5 > gpurun_out/exp6/cold_c5.log 2>&1; tail -1 gpurun_out/exp6/cold_c5.log

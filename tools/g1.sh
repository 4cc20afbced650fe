set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/g1
timeout -k 10 900 python -u -m pytest tests/test_gpu_api_surface.py tests/test_gpu_golden.py tests/test_gpu_pins.py tests/test_gpu_distributed.py tests/test_bench_launch.py -m gpu -v --timeout 500 --timeout-method thread > gpurun_out/g1/tests.log 2>&1 || true
grep -E "passed|failed|PASSED|FAILED|ERROR" gpurun_out/g1/tests.log | tail -80
timeout -k 10 180 python tools/pmc_trace.py --config c3 --out gpurun_out/g1/r04_trace_c3_pmc.json > gpurun_out/g1/pmc.log 2>&1
python -c "import json;d=json.load(open('gpurun_out/g1/r04_trace_c3_pmc.json'));[print(k,v.get('median_s'),v.get('f64_valu_share'),v['per_launch'].get('SQ_INSTS_VALU'),v['per_launch'].get('SQ_INSTS_SALU')) for k,v in d['kernels'].items()]"
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so timeout -k 10 180 python tools/trace_phases.py c3 > gpurun_out/g1/phases_c3.json 2> gpurun_out/g1/phases.err
cat gpurun_out/g1/phases_c3.json

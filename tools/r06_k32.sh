#!/bin/bash
# Round 6: 32-bit sort keys in the trace kernel — CSR parity (golden / construction / full size),
# then the count-pass A/B against the 64-bit-key variant (k64), then VALU counters of both at C3.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_construct.py tests/test_gpu_fullsize.py tests/test_gpu_reference_suite.py -x -q --timeout 300 --timeout-method thread > $O/k32_tests.log 2>&1
tail -1 $O/k32_tests.log
bash tools/trace_ab.sh r06/k32_ab k64 c2 c5 c3
timeout -k 10 200 python tools/pmc_trace.py --config c3 --out $O/r06_trace_c3_pmc.json > /dev/null 2> $O/pmc_k32.err
SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_k64.so timeout -k 10 200 python tools/pmc_trace.py --config c3 --out $O/r06_trace_c3_pmc_k64.json > /dev/null 2>> $O/pmc_k32.err

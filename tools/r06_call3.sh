#!/bin/bash
# Round 6: dense output ranges for the time-paired adjoint (C4): parity tests, bench, PMC;
# the C4 adjoint with geometry columns (SPHRT_TCOLS=geom: no per-call gather of y).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_fullsize.py tests/test_gpu_properties.py -x -q --timeout 300 --timeout-method thread -k "dynamic or c4" > $O/dense_tests.log 2>&1
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 100 > $O/bench_c4_dense.json 2> $O/bench_c4_dense.err
SPHRT_TCOLS=geom timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 100 > $O/bench_c4_dense_geomcols.json 2>/dev/null
timeout -k 10 400 python tools/pmc_forward.py --config c4 --adjoint --out $O/r06_adjoint_c4_pmc_dense.json --workdir $O/pmc_adj2 > $O/pmc_adj2.log 2>&1

#!/bin/bash
# Round 6: C4 first construction after the broadcast fix; C4 forward / time-paired gradient
# kernel split (rocprofv3 kernel trace of the C4 bench) and their PMC records.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 120 python tools/first_construct.py --warm c2 --config c4 > $O/first_c4_fixed.json 2>&1
timeout -k 10 120 python tools/first_construct.py --warm none --config c4 > $O/first_c4_nowarm_fixed.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bench_c4 -o run --output-format csv -- python bench.py --config c4 --no-cpu-baseline --steps 100 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 400 python tools/pmc_forward.py --config c4 --adjoint --out $O/r06_adjoint_c4_pmc.json --workdir $O/pmc_adj > $O/pmc_adj.log 2>&1
timeout -k 10 400 python tools/pmc_forward.py --config c4 --out $O/r06_forward_c4_pmc.json --workdir $O/pmc_fwd > $O/pmc_fwd.log 2>&1

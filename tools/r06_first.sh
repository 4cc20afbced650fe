#!/bin/bash
# Round 6, first GPU call: where the first dynamic Operator's time goes, and the new roofline.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
timeout -k 10 180 python tools/first_construct.py --warm c2 --config c4 --profile > $O/first_c4.json 2> $O/first_c4.err
timeout -k 10 120 python tools/first_construct.py --warm none --config c4 > $O/first_c4_nowarm.json 2>&1
timeout -k 10 120 python tools/first_construct.py --warm c2 --config c5 > $O/first_c5.json 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_first_c4 -o run --output-format csv -- python tools/first_construct.py --warm c2 --config c4 > $O/first_c4_prof.json 2>&1
timeout -k 10 300 python bench.py --no-strong-legs > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 400 python tools/pmc_forward.py --config c4 --adjoint --out $O/r06_adjoint_c4_pmc.json --workdir $O/pmc_adj > $O/pmc_adj.log 2>&1
timeout -k 10 400 python tools/pmc_forward.py --config c4 --out $O/r06_forward_c4_pmc.json --workdir $O/pmc_fwd > $O/pmc_fwd.log 2>&1

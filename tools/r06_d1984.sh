#!/bin/bash
# Round 6: dense blocks of 1984 (the tree): the gpu suite, the dense output stage of 2560 (tree)
# against 2816 / 3072 (variants) on the C4 adjoint, then the C4 bench line.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/d1984_gpu_tests.log 2>&1
tail -1 $O/d1984_gpu_tests.log
for r in 1 2 3; do
  for v in tree o2816 o3072; do
    lib=""; [ $v != tree ] && lib=sph_raytracer_amd/lib/variants/libsphrt_$v.so
    SPHRT_LIB=$lib timeout -k 10 120 python tools/adjoint_stats.py --config c4 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'v': '$v', 'r': $r, 'config': 'c4', 'adjoint_kernel_us': d['adjoint_kernel_us'], 'forward_us': d['forward_us']}))" >> $O/r06_ostage1984_ab.jsonl
  done
done
cat $O/r06_ostage1984_ab.jsonl
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/r06_bench_c4_d1984.json 2> $O/bench_c4_d1984.err
python -c "import json; d=json.load(open('$O/r06_bench_c4_d1984.json')); print('c4 fwd', d['ms_per_step'], 'adj', d['adjoint']['ms_per_step'], 'ratio', d['adjoint']['ms_per_step']/d['ms_per_step'])"

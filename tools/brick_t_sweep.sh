set -e
mkdir -p gpurun_out
for c in c3 c5; do
 for b in off 1,4,8 1,2,8 1,4,4 2,2,8; do
  (export SPHRT_BRICK_T=$b; timeout -k 10 200 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline 2>/dev/null) | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'config':'$c','brick_t':'$b','fwd_us':d['ms_per_step']*1e3,'adj_us':d['adjoint']['ms_per_step']*1e3}))" >> gpurun_out/tsweep.jsonl
  echo "$c $b"
 done
done

# Brick-shape sweep of the staged forward: tools/prof_forward.py per config under SPHRT_BRICK.
#   bash tools/brick_sweep.sh "c5 c3" "2,4,4 4,2,4" [SPHRT_BRICK_T]   -> gpurun_out/brick_sweep.jsonl
# (the third argument names the variable: SPHRT_BRICK, the default, or SPHRT_BRICK_T)
set -e
mkdir -p gpurun_out
for c in ${1:-c5 c3 c4}; do
  for b in ${2:-2,4,4 2,2,8 4,4,2 1,4,8 4,2,4}; do
    (export "${3:-SPHRT_BRICK}=$b"; timeout -k 10 120 python tools/prof_forward.py --config $c --rounds 3 2>/dev/null) | sed "s/}$/, \"config\": \"$c\", \"brick\": \"$b\", \"var\": \"${3:-SPHRT_BRICK}\"}/" >> gpurun_out/brick_sweep.jsonl
    echo "$c $b done"
  done
done

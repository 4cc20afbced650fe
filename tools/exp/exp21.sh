set -e
export TMPDIR=/tmp
SPHRT_BENCH_ONE_DEVICE=1 SPHRT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -20 gpurun_out/bench_n2.err; exit 1; }
cut -c1-400 gpurun_out/bench_n2.json
grep -o '"final_gather": {[^}]*}' gpurun_out/bench_n2.json

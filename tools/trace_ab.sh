#!/bin/bash
# Trace count-pass A/B (HIP events, tools/trace_time.py) of the product library against a variant
# (default: lib/variants/libsphrt_base.so from tools/build_ab.py), interleaved, then the exact-path
# and sort-fallback counters; stops at the first failure.
#   bash tools/trace_ab.sh <out-dir> [variant-name] [configs...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/$1; var=${2:-base}; shift 2
cfgs=${@:-c2 c5 c4 c3}
mkdir -p "$out"
for rep in 1 2; do
  for c in $cfgs; do
    SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_$var.so timeout -k 10 120 python tools/trace_time.py $c >> "$out/ab.jsonl" || exit 1
    timeout -k 10 120 python tools/trace_time.py $c >> "$out/ab.jsonl" || exit 1
  done
done
cat "$out/ab.jsonl"
timeout -k 10 180 python tools/exact_stats.py $cfgs | tee "$out/exact_stats.jsonl"

set -e
for c in c3 c5 c2; do bash tools/ab_variants.sh $c "trace_kernel" base swz; done

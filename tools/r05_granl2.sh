#!/bin/bash
# C3 forward ablation: every granule DMA of the table-mode forward redirected
# to one L2-resident 16/32 KB tile (variant libsphrt_granl2: results wrong, timing only).  If the
# kernel time does not drop, the 0.21 GB of density-granule fills above the CSR stream are not
# what bounds it.  Interleaved base / variant rounds in one call; PMC FETCH/WRITE of both.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/granl2; mkdir -p $O
V=sph_raytracer_amd/lib/variants/libsphrt_granl2.so
for i in 1 2; do
  timeout -k 10 180 python tools/prof_forward.py --config c3 --rounds 3 > $O/base_$i.json
  SPHRT_LIB=$V timeout -k 10 180 python tools/prof_forward.py --config c3 --rounds 3 > $O/var_$i.json
done
cat $O/base_*.json $O/var_*.json | cut -c1-400
timeout -k 10 300 python tools/pmc_forward.py --config c3 --out $O/base_pmc.json > $O/base_pmc.log 2>&1
SPHRT_LIB=$V timeout -k 10 300 python tools/pmc_forward.py --config c3 --out $O/var_pmc.json > $O/var_pmc.log 2>&1
head -c 600 $O/base_pmc.json; echo; head -c 600 $O/var_pmc.json

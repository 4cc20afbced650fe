set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/check gpurun_out/stamps
timeout -k 10 120 python tools/exact_stats.py > gpurun_out/stamps/exact_stats.jsonl 2>&1 || { cat gpurun_out/stamps/exact_stats.jsonl; exit 1; }
cat gpurun_out/stamps/exact_stats.jsonl
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/check/tests.log 2>&1 || { tail -30 gpurun_out/check/tests.log; exit 1; }
grep "per view" gpurun_out/check/tests.log || true
tail -2 gpurun_out/check/tests.log
bash tools/ab_variants.sh c3 "exact_wave" ex1
bash tools/ab_variants.sh c5 "exact_wave" ex1
for c in c3 c5; do
  SPHRT_LIB=sph_raytracer_amd/lib/variants/libsphrt_tstamps.so timeout -k 10 180 python tools/exact_phases.py $c > gpurun_out/stamps/${c}_tstamps.json 2> gpurun_out/stamps/${c}_tstamps.err
  echo "$c $(cat gpurun_out/stamps/${c}_tstamps.json)"
done

set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tabpmc
timeout -k 10 120 python tools/pmc_trace.py --config c3 --match local_table_radix --counters FETCH_SIZE --out gpurun_out/tabpmc/r04_table_c3_pmc_fetch.json > gpurun_out/tabpmc/b.log 2>&1
timeout -k 10 120 python tools/pmc_trace.py --config c3 --match local_table_radix --counters WRITE_SIZE --out gpurun_out/tabpmc/r04_table_c3_pmc_write.json > gpurun_out/tabpmc/c.log 2>&1
timeout -k 10 120 python tools/pmc_trace.py --config c3 --match screen_kernel --out gpurun_out/tabpmc/r04_screen_c3_pmc.json > gpurun_out/tabpmc/d.log 2>&1
for f in gpurun_out/tabpmc/*.json; do python -c "import json;d=json.load(open('$f'));[print('$f',k,v.get('median_s'),{c:round(x/1e6,2) for c,x in v['per_launch'].items()}) for k,v in d['kernels'].items()]"; done

set -e
export TMPDIR=/tmp
for v in a1 a2 a3 a4 full; do
rm -rf gpurun_out/apmc_$v
L=sph_raytracer_amd/lib/variants/libsphrt_$v.so; [ $v = full ] && L=sph_raytracer_amd/lib/libsphrt.so
SPHRT_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -d gpurun_out/apmc_$v -o p --output-format csv -- python tools/trace_bench.py c2 --reps 1 > gpurun_out/apmc_$v.log 2>&1 || echo "fail $v"
done

#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE calibration for 2/4/8/16-byte lanes and the table build's
# 4+8-byte pair (tools/fetch_calib), then PMC passes over the C3 table kernel (construction).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o calib --output-format csv -- tools/fetch_calib > $O/calib.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o calib --output-format csv -- tools/fetch_calib >> $O/calib.log 2>&1
timeout -s KILL 60 rocprofv3 --kernel-trace -d $O/calib_trace -o calib --output-format csv -- tools/fetch_calib >> $O/calib.log 2>&1
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES" "SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_INSTS_LDS"; do
  tag=$(echo $c | cut -d, -f1 | tr A-Z a-z)
  timeout -k 10 120 python tools/pmc_trace.py --config c3 --counters $c --match local_table --out $O/r06_table_c3_pmc_$tag.json > /dev/null 2> $O/pmc_table_$tag.err
done
ls $O/r06_table_c3_pmc_*

#!/bin/bash
# Kernel A/B of Operator construction between environment settings of the in-tree library:
#   bash tools/ab_env.sh CONFIG NAME1="ENV=V ..." NAME2="ENV=V ..." ...
# rocprofv3 kernel stats of tools/operator_time.py per setting into gpurun_out/ab/CONFIG_NAME_*.
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
C=$1; shift
O=gpurun_out/ab; mkdir -p $O
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${C}_$name -o run --output-format csv -- python tools/operator_time.py --config $C --reps 5 > $O/op_${C}_$name.json 2>$O/op_${C}_$name.err
  f=$(find $O/prof_${C}_$name -name "*kernel_stats.csv"); cp $f $O/${C}_${name}_kernel_stats.csv
  echo "== $name ($envs) $(cat $O/op_${C}_$name.json)"
done

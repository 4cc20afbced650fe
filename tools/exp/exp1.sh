set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/exp1
timeout -k 10 300 python tools/fwd_study.py --config c3 > gpurun_out/exp1/study_c3.log 2>&1
cat gpurun_out/exp1/study_c3.log
timeout -k 10 120 python tools/fwd_study.py --config c2 --reps 50 > gpurun_out/exp1/study_c2.log 2>&1
cat gpurun_out/exp1/study_c2.log
for c in c2 c5 c3; do timeout -k 10 300 python tools/prof_forward.py --config $c > gpurun_out/exp1/apply_$c.log 2>&1; cat gpurun_out/exp1/apply_$c.log; done
timeout -k 10 300 python tools/pmc_forward.py --config c3 --reps 5 --out gpurun_out/exp1/pmc_c3.json > gpurun_out/exp1/pmc_c3.log 2>&1
tail -c 800 gpurun_out/exp1/pmc_c3.log

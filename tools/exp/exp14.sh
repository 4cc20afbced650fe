set -e
export TMPDIR=/tmp
timeout -k 10 300 python tools/fwd_study.py --config c5 2>&1 | grep -v amdgpu

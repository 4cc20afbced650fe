set -e
export TMPDIR=/tmp
timeout -k 10 120 python tools/prelude_time.py c3
timeout -k 10 120 python tools/prelude_time.py c2

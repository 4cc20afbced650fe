set -e
export TMPDIR=/tmp
bash tools/ab_variants.sh c3 "local_table" tw7 tw10
bash tools/ab_variants.sh c3 "local_table" tw7 tw10

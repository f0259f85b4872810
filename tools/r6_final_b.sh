# Round-6 final build, part 2: C5 and C4 measured, then the multi-GPU shard projections of every config
set -o pipefail
CONFIGS="C5 C4" bash tools/r6_measure.sh || exit 1
NOTESTS=1 CONFIGS="C2 C3 C5 C4" bash tools/r6_shards.sh

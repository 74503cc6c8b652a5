#!/bin/bash
# round 4, final tree: per-rank step at N = 1 / 2 / 4 / 8 (rank 0's shard scored alone into pinned arrays,
# tools/shard_step_ab.py), three rounds x 30 steps, the §5 pricing table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04sf}
mkdir -p $OUT
SHARD_AB_NS=1,2,4,8 timeout -k 10 300 python -u tools/shard_step_ab.py 3 30 > $OUT/shards.json 2> $OUT/shards.err || { echo "shards failed"; tail -30 $OUT/shards.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/shards.json'))
for r in d['results']: print(r['ranks'], r['shard_pairs'], r['median_ms'], r['min_ms'], r['max_ms'])"

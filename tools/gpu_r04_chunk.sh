#!/bin/bash
# round 4: packed chunk size at the target point after the pool rewrite (N = 1 and rank shards), one engine per
# setting and size, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04c2}
mkdir -p $OUT
SHARD_AB_SETTINGS="default=;c2m=OVL_PIPE_CHUNK:2000000;c700k=OVL_PIPE_CHUNK:700000;c500k=OVL_PIPE_CHUNK:500000;c350k=OVL_PIPE_CHUNK:350000" SHARD_AB_NS=1,2,4 timeout -k 10 500 python -u tools/shard_step_ab.py 4 30 > $OUT/chunk_ab.json 2> $OUT/chunk_ab.err || { echo "chunk ab failed"; tail -30 $OUT/chunk_ab.err; exit 1; }
echo "chunk ab ok"

#!/bin/bash
# round 5: per-rank step A/B (tools/shard_step_ab.py) under SHARD_AB_SETTINGS, at OVL_POOL_THREADS 12 and 15
# usage: bash tools/gpu_r05_ab.sh <tag> "<settings>" [Ns]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1
mkdir -p $OUT
for T in 12 15; do
  OVL_POOL_THREADS=$T SHARD_AB_SETTINGS="$2" SHARD_AB_NS=${3:-1,2,4,8} timeout -k 10 300 python3 -u tools/shard_step_ab.py 3 30 \
    > $OUT/ab_t$T.json 2> $OUT/ab_t$T.err || { echo "ab t$T failed"; tail -30 $OUT/ab_t$T.err; exit 1; }
done
echo "all ok"

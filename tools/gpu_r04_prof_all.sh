#!/bin/bash
# round 4: profiles of the default bench workload and of rank 0's shard at N = 2 and N = 8 (bench.py --shard)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r04prof}
bash tools/gpu_r04_profile.sh target ${TAG}_target || exit 1
SHARD=0/2 bash tools/gpu_r04_profile.sh target ${TAG}_shard0of2 || exit 1
SHARD=0/8 bash tools/gpu_r04_profile.sh target ${TAG}_shard0of8 || exit 1
echo "all profiles ok"

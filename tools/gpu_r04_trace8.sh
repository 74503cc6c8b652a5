#!/bin/bash
# round 4: pipeline trace (OVL_TRACE_PIPE=1) of the per-rank step at N = 1 and N = 8 (rank 0's shard), final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04t8}
mkdir -p $OUT
SHARD_AB_NS=1,8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 2 20 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "trace ok"; cat $OUT/trace.json

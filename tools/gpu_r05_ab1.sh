#!/bin/bash
# round 5: per-rank step, default pipeline vs every pair packed (no direct int32 chunk), N = 1/2/4/8, under a kernel
# trace (the gaps between a call's kernels), then the pipeline trace of the all-packed N = 8 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r05ab1}
mkdir -p $OUT
export TMPDIR=/tmp
SHARD_AB_SETTINGS="default=;packed=OVL_PACK_DIRECT_PCT:0" SHARD_AB_NS=1,2,4,8 timeout -k 10 300 \
  rocprofv3 --kernel-trace -d $OUT/prof -o ab -- python3 -u tools/shard_step_ab.py 3 30 > $OUT/ab.json 2> $OUT/ab.err \
  || { echo "ab failed"; tail -30 $OUT/ab.err; exit 1; }
echo "ab ok"
SHARD_AB_SETTINGS="packed=OVL_PACK_DIRECT_PCT:0" SHARD_AB_NS=8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 2 20 \
  > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "all ok"

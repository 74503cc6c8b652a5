#!/bin/bash
# round 5: per-rank steps (tools/shard_step_ab.py, rank 0's shard scored alone) of the target list and of cfg4 (BASELINE
# configs[3]) at N = 1/2/4/8, the cfg4 shards' kernels under a kernel trace, and the target's pipeline trace at N = 1, 8
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r05shards}
mkdir -p $OUT
export TMPDIR=/tmp
SHARD_AB_NS=1,2,4,8 timeout -k 10 300 python3 -u tools/shard_step_ab.py 3 30 > $OUT/target.json 2> $OUT/target.err \
  || { echo "target failed"; tail -30 $OUT/target.err; exit 1; }
echo "target ok"
SHARD_AB_CONFIG=cfg4 SHARD_AB_NS=1,2,4,8 timeout -k 10 400 python3 -u tools/shard_step_ab.py 3 10 > $OUT/cfg4.json \
  2> $OUT/cfg4.err || { echo "cfg4 failed"; tail -30 $OUT/cfg4.err; exit 1; }
echo "cfg4 ok"
SHARD_AB_CONFIG=cfg4 SHARD_AB_NS=1,2,4,8 OVL_TRACE_PIPE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt4 \
  -o kt4 -- python3 -u tools/shard_step_ab.py 1 10 > $OUT/cfg4_kt.json 2> $OUT/cfg4_kt.err || { echo "cfg4 kt failed"; tail -30 $OUT/cfg4_kt.err; exit 1; }
echo "cfg4 kt ok"
SHARD_AB_NS=1,8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 2 20 > $OUT/trace.json \
  2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "all ok"

#!/bin/bash
# round 5 baseline on one box: kernel time against call size (HBM vs host-packed outputs, rocprofv3 kernel
# trace), per-rank steps at N = 1/2/4/8, and the pipeline trace of the N = 1 and N = 8 steps
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r05base}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o size -- python3 -u tools/size_probe.py 20 \
  > $OUT/size.json 2> $OUT/size.err || { echo "size probe failed"; tail -30 $OUT/size.err; exit 1; }
echo "size ok"
SHARD_AB_NS=1,2,4,8 timeout -k 10 300 python -u tools/shard_step_ab.py 3 30 > $OUT/shards.json 2> $OUT/shards.err \
  || { echo "shards failed"; tail -30 $OUT/shards.err; exit 1; }
echo "shards ok"
SHARD_AB_NS=1,8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 2 20 > $OUT/trace.json \
  2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "all ok"

#!/bin/bash
# round 5: streamed records, out-of-order expansion -- transport tests, per-rank steps rec vs 2-byte packing under
# a kernel trace, then the pipeline trace at N = 1 and 8
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r05stream2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py \
  tests/test_gpu_compact_pairs.py tests/test_gpu_parity.py -m gpu > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SHARD_AB_SETTINGS="rec=;r10=OVL_PACK_DIRECT_PCT:10;pk2=OVL_PACK:1" SHARD_AB_NS=1,2,4,8 timeout -k 10 300 python3 -u tools/shard_step_ab.py 3 30 \
  > $OUT/ab.json 2> $OUT/ab.err || { echo "ab failed"; tail -30 $OUT/ab.err; exit 1; }
echo "ab ok"
SHARD_AB_SETTINGS="rec=" SHARD_AB_NS=1,8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 2 20 \
  > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
SHARD_AB_SETTINGS="rec=" SHARD_AB_NS=1,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt \
  -- python3 -u tools/shard_step_ab.py 2 20 > $OUT/kt.json 2> $OUT/kt.err || { echo "kt failed"; tail -30 $OUT/kt.err; exit 1; }
echo "all ok"

#!/bin/bash
# round 5: streamed tile records (OVL_PACK=2, default) -- the GPU tests that cover the transport, then the
# per-rank steps against 2-byte packing expanded after each chunk (OVL_PACK=1), and the pipeline trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r05stream}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py \
  tests/test_gpu_compact_pairs.py tests/test_gpu_parity.py -m gpu > $OUT/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SHARD_AB_SETTINGS="rec=;pk2=OVL_PACK:1" SHARD_AB_NS=1,2,4,8 timeout -k 10 300 python3 -u tools/shard_step_ab.py 3 30 \
  > $OUT/ab.json 2> $OUT/ab.err || { echo "ab failed"; tail -30 $OUT/ab.err; exit 1; }
echo "ab ok"
SHARD_AB_SETTINGS="rec=" SHARD_AB_NS=1,8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 2 20 \
  > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "all ok"

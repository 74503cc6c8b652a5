#!/bin/bash
# round 4 (record of a rejected experiment; the knob and sink 3 were removed after it): one launch over a call's
# chunks (OVL_ONE_LAUNCH=1) against a launch per chunk, per-rank step
# at N = 1 / 2 / 4 / 8, one engine per setting and size, interleaved; traced once
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04o}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q -k "one_launch or step_transport" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SHARD_AB_SETTINGS="one=;per_chunk=OVL_ONE_LAUNCH:0" SHARD_AB_NS=1,2,4,8 timeout -k 10 400 python -u tools/shard_step_ab.py 5 30 > $OUT/one_ab.json 2> $OUT/one_ab.err || { echo "one ab failed"; tail -30 $OUT/one_ab.err; exit 1; }
echo "one ab ok"
SHARD_AB_SETTINGS="one=;per_chunk=OVL_ONE_LAUNCH:0" SHARD_AB_NS=1,2 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 1 3 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "trace ok"

#!/bin/bash
# round 4: streamed cycle removal, the tree's dict builder (progressive successor rows) against the previous ones
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04s}
mkdir -p $OUT
OVL_TRACE_STREAM=1 timeout -k 10 400 python -u tools/stream_ab.py 5 > $OUT/stream_ab.json 2> $OUT/stream_ab.err || { echo "stream ab failed"; tail -30 $OUT/stream_ab.err; exit 1; }
cat $OUT/stream_ab.json
grep ovl_stream $OUT/stream_ab.err | tail -6

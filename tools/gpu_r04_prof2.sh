#!/bin/bash
# round 4: the cycle-removal A/B with the stream trace (replay alone, replay then dicts, streamed without and with
# the component helper), then the target profiles (kernel trace + stats, four PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04p}
mkdir -p $OUT
OVL_TRACE_STREAM=1 timeout -k 10 400 python -u tools/replay_ab.py 5 > $OUT/replay_ab.json 2> $OUT/replay_ab.err || { echo "replay ab failed"; tail -30 $OUT/replay_ab.err; exit 1; }
echo "replay ab ok"
grep ovl_stream $OUT/replay_ab.err | tail -6
bash tools/gpu_r04_profile.sh target ${1:-r04p}_target || exit 1
echo "profiles ok"

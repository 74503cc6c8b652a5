#!/bin/bash
# round 4: the IX path diagnostic, then the A/Bs of gpu_r04_mix1.sh (shard step, replay, one-shot timeline) and
# gpu_r04_mix2.sh (banded tests, band A/B, lane probe)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04e}
mkdir -p $OUT
timeout -k 10 120 python -u tools/ix_diag.py > $OUT/ix_diag.txt 2>&1 || { echo "ix diag failed"; tail -20 $OUT/ix_diag.txt; exit 1; }
cat $OUT/ix_diag.txt
bash tools/gpu_r04_shard_ab.sh ${1:-r04e} || exit 1
timeout -k 10 400 python -u tools/replay_ab.py 5 > $OUT/replay_ab.json 2> $OUT/replay_ab.err || { echo "replay ab failed"; tail -30 $OUT/replay_ab.err; exit 1; }
echo "replay ab ok"
OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/one_shot_timeline.py 20 > $OUT/one_shot.txt 2> $OUT/one_shot_trace.txt || { echo "one-shot timeline failed"; tail -20 $OUT/one_shot_trace.txt; exit 1; }
cat $OUT/one_shot.txt
bash tools/gpu_r04_mix2.sh ${1:-r04e} || exit 1

#!/bin/bash
# round 4, second A/B batch: the compact-pair tests alone (the IX path), the per-rank step at the shard sizes of
# N = 1 / 2 / 4 / 8 with the packed-chunk ramp and finer host expansion parts (one engine per setting and size),
# traced; the one-shot timeline; the replay with the prefetch / 12-byte records against the previous build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04f}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact_pairs.py -x -v --timeout 120 --timeout-method thread > $OUT/compact_tests.log 2>&1 || { echo "compact tests failed"; tail -40 $OUT/compact_tests.log; exit 1; }
tail -3 $OUT/compact_tests.log
export SHARD_AB_SETTINGS="default=;noramp=OVL_PACK_RAMP:0;part64k=OVL_EXPAND_PART:65536;before=OVL_PACK_RAMP:0,OVL_EXPAND_PART:65536;pm64k=OVL_PACK_MIN:65536;pm64k_d10=OVL_PACK_MIN:65536,OVL_PACK_DIRECT_PCT:10;d10=OVL_PACK_DIRECT_PCT:10"
timeout -k 10 500 python -u tools/shard_step_ab.py 4 30 > $OUT/shard_ab.json 2> $OUT/shard_ab.err || { echo "ab failed"; tail -30 $OUT/shard_ab.err; exit 1; }
echo "ab ok"
SHARD_AB_SETTINGS="default=;pm64k=OVL_PACK_MIN:65536" OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 1 3 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "trace ok"
OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/one_shot_timeline.py 20 > $OUT/one_shot.txt 2> $OUT/one_shot_trace.txt || { echo "one-shot timeline failed"; tail -20 $OUT/one_shot_trace.txt; exit 1; }
cat $OUT/one_shot.txt
timeout -k 10 400 python -u tools/replay_ab.py 5 > $OUT/replay_ab.json 2> $OUT/replay_ab.err || { echo "replay ab failed"; tail -30 $OUT/replay_ab.err; exit 1; }
echo "replay ab ok"

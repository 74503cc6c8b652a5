#!/bin/bash
# round 4: per-rank step at the shard sizes of N = 2 / 4 / 8 (tools/shard_step_ab.py), pipeline settings
# interleaved; then one traced call per shard size (OVL_TRACE_PIPE=1: microsecond offsets of the pipeline events)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
export SHARD_AB_SETTINGS="${SHARD_AB_SETTINGS:-default=;pack64k=OVL_PACK_MIN:65536;pack64k_d0=OVL_PACK_MIN:65536,OVL_PACK_DIRECT_PCT:0;pack64k_d10=OVL_PACK_MIN:65536,OVL_PACK_DIRECT_PCT:10;pack64k_d25=OVL_PACK_MIN:65536,OVL_PACK_DIRECT_PCT:25;pack64k_c256k=OVL_PACK_MIN:65536,OVL_PIPE_CHUNK:262144;int32=OVL_PACK:0}"
timeout -k 10 400 python -u tools/shard_step_ab.py 5 30 > $OUT/shard_ab.json 2> $OUT/shard_ab.err || { echo "ab failed"; tail -30 $OUT/shard_ab.err; exit 1; }
echo "ab ok"
SHARD_AB_SETTINGS="default=;pack64k=OVL_PACK_MIN:65536" OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 1 3 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "trace ok"

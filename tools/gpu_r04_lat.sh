#!/bin/bash
# round 4: uniform_kernel's latency mode (two wavefronts per tile) up to 8 (default) / 16 / 32 / 64 tiles per CU, at
# the shard sizes of N = 2 / 4 / 8 and the whole list, one engine per setting and size, interleaved; traced once
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04l}
mkdir -p $OUT
SHARD_AB_SETTINGS="default=;lat16=OVL_LAT_TILES:16;lat32=OVL_LAT_TILES:32;lat64=OVL_LAT_TILES:64" SHARD_AB_NS=1,2,4,8 timeout -k 10 500 python -u tools/shard_step_ab.py 4 30 > $OUT/lat_ab.json 2> $OUT/lat_ab.err || { echo "lat ab failed"; tail -30 $OUT/lat_ab.err; exit 1; }
echo "lat ab ok"
SHARD_AB_SETTINGS="default=;lat16=OVL_LAT_TILES:16;lat32=OVL_LAT_TILES:32" SHARD_AB_NS=4,8 OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 1 3 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "trace ok"

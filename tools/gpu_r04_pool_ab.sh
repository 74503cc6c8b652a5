#!/bin/bash
# round 4: the lock-free pool dispatch (ovl_pool.h) against the previous build (build/ab_prev/libovl.so), with and
# without the packed-chunk ramp, per-rank step at the shard sizes of N = 1 / 2 / 4 / 8; the pool probe; the
# pipeline / compact / resident-read GPU tests on the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04g}
mkdir -p $OUT
timeout -k 10 60 genome-assembly-using-overlap-graphs_amd/build/pool_probe 3000 > $OUT/pool_probe.txt 2>&1 || { echo "probe failed"; cat $OUT/pool_probe.txt; exit 1; }
cat $OUT/pool_probe.txt
# (an assertion failure here is recorded and the A/Bs still run; a crash or time-out ends the script)
OVL_TRACE_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_compact_pairs.py tests/test_gpu_reads_resident.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests ended with $rc"; exit 1; }
SHARD_AB_SETTINGS="noramp=OVL_PACK_RAMP:0;ramp=" OVL_LIB_PATH=genome-assembly-using-overlap-graphs_amd/build/ab_prev/libovl.so timeout -k 10 300 python -u tools/shard_step_ab.py 3 30 > $OUT/shard_prev.json 2> $OUT/shard_prev.err || { echo "ab prev failed"; tail -30 $OUT/shard_prev.err; exit 1; }
echo "prev ok"
SHARD_AB_SETTINGS="noramp=OVL_PACK_RAMP:0;ramp=;noramp_p64=OVL_PACK_RAMP:0,OVL_EXPAND_PART:65536;pm64k=OVL_PACK_MIN:65536,OVL_PACK_RAMP:0" timeout -k 10 400 python -u tools/shard_step_ab.py 3 30 > $OUT/shard_new.json 2> $OUT/shard_new.err || { echo "ab new failed"; tail -30 $OUT/shard_new.err; exit 1; }
echo "new ok"
SHARD_AB_SETTINGS="noramp=OVL_PACK_RAMP:0;ramp=;pm64k=OVL_PACK_MIN:65536,OVL_PACK_RAMP:0" OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/shard_step_ab.py 1 3 > $OUT/trace.json 2> $OUT/trace.err || { echo "trace failed"; tail -30 $OUT/trace.err; exit 1; }
echo "trace ok"
OVL_TRACE_STREAM=1 timeout -k 10 400 python -u tools/replay_ab.py 5 > $OUT/replay_ab.json 2> $OUT/replay_ab.err || { echo "replay ab failed"; tail -30 $OUT/replay_ab.err; exit 1; }
echo "replay ab ok"

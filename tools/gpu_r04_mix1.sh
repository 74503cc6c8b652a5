#!/bin/bash
# round 4: the GPU tests of the files the knob removal touched, then the shard-size step A/B and the
# cycle-removal A/B (replay and surviving-edge dicts)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04d}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dp_lane.py tests/test_gpu_pipeline.py tests/test_gpu_compact_pairs.py tests/test_gpu_c_abi.py tests/test_gpu_reads_resident.py tests/test_gpu_bench_dist.py tests/test_gpu_assembly.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_r04_shard_ab.sh ${1:-r04d} || exit 1
timeout -k 10 400 python -u tools/replay_ab.py 5 > $OUT/replay_ab.json 2> $OUT/replay_ab.err || { echo "replay ab failed"; tail -30 $OUT/replay_ab.err; exit 1; }
echo "replay ab ok"
OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/one_shot_timeline.py 20 > $OUT/one_shot.txt 2> $OUT/one_shot_trace.txt || { echo "one-shot timeline failed"; tail -20 $OUT/one_shot_trace.txt; exit 1; }
cat $OUT/one_shot.txt
bash tools/gpu_r04_mix2.sh ${1:-r04d} || exit 1

#!/bin/bash
# round 4: kernel-exact launch timing (hipExtLaunchKernelGGL events) -- the timing tests and a default bench line;
# the streamed cycle-removal A/B (progressive predecessor dicts against the previous builder); the shard profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04m}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_bench_dist.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench ok"
OVL_TRACE_STREAM=1 timeout -k 10 300 python -u tools/stream_ab.py 5 > $OUT/stream_ab.json 2> $OUT/stream_ab.err || { echo "stream ab failed"; tail -30 $OUT/stream_ab.err; exit 1; }
cat $OUT/stream_ab.json
SHARD=0/2 bash tools/gpu_r04_profile.sh target ${1:-r04m}_shard0of2 || exit 1
SHARD=0/8 bash tools/gpu_r04_profile.sh target ${1:-r04m}_shard0of8 || exit 1
echo "profiles ok"

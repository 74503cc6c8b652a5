#!/bin/bash
# round 3 quick check: the named test files (default: all GPU tests), then the default bench without the CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r03q}
shift
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err \
  || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench ok"

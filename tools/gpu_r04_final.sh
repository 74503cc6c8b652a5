#!/bin/bash
# round 4, end of round on one box: every GPU test, smoke, the default bench line (N = 1, CPU baseline), the N = 2
# rehearsal and the target profile (kernel trace + PMC) of the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r04z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
  || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench ok"
timeout -k 10 500 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/n2.json 2> $OUT/n2.err \
  || { echo "n2 failed"; tail -30 $OUT/n2.err; exit 1; }
echo "n2 ok"
bash tools/gpu_r04_profile.sh target ${TAG}_target || exit 1
echo "all ok"

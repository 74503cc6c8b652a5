#!/bin/bash
# round 4: the driver's round-end tier on one box -- every GPU test, smoke, the default bench line (N = 1, with
# the CPU baseline), the processes left after it, and the N = 2 line (both ranks on GPU 0, gloo)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04t}
mkdir -p $OUT
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
  || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench ok"
sleep 2
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $OUT/ps_after.txt
ls /dev/shm > $OUT/shm_after.txt 2>&1
timeout -k 10 500 python -u bench.py --gpus 2 --steps 20 --warmup 5 > $OUT/n2.json 2> $OUT/n2.err \
  || { echo "n2 failed"; tail -30 $OUT/n2.err; exit 1; }
echo "n2 ok"

#!/bin/bash
# round 2: the round-end tiers (all GPU tests, smoke, default bench), the processes left after bench exits,
# and the N=2 flow rehearsal (gloo, both ranks on the one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $OUT/ps_before.txt
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
  || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench ok"
sleep 2
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > $OUT/ps_after.txt
diff $OUT/ps_before.txt $OUT/ps_after.txt | grep -v " ps -u" || true
OVL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 \
  > $OUT/rehearse_n2.json 2> $OUT/rehearse_n2.err || { echo "rehearsal failed"; tail -30 $OUT/rehearse_n2.err; exit 1; }
cat $OUT/rehearse_n2.json

#!/bin/bash
# round 2: the round-end tiers (all GPU tests, smoke, default bench) plus the N=2 flow rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/r02/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r02/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -30 gpurun_out/r02/smoke.log; exit 1; }
tail -1 gpurun_out/r02/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err \
  || { echo "bench failed"; tail -30 gpurun_out/r02/bench.err; exit 1; }
echo "bench ok"
OVL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 \
  > gpurun_out/r02/rehearse_n2.json 2> gpurun_out/r02/rehearse_n2.err || { echo "rehearsal failed"; tail -30 gpurun_out/r02/rehearse_n2.err; exit 1; }
cat gpurun_out/r02/rehearse_n2.json

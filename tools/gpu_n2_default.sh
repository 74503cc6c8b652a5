#!/bin/bash
# round 3: the driver's N > 1 command shapes on the one-GPU box (2 ranks share GPU 0; flow and wall time, not
# a scaling number): bench.py --gpus 2 with its own launcher, and under torch.distributed.run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r03r}
mkdir -p $OUT
s=$(date +%s)
timeout -k 10 500 python -u bench.py --gpus 2 --steps 50 --warmup 5 > $OUT/n2_self.json 2> $OUT/n2_self.err || { echo "self-launch failed"; tail -20 $OUT/n2_self.err; exit 1; }
echo "self-launched N=2: $(( $(date +%s) - s )) s"
s=$(date +%s)
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 50 --warmup 5 > $OUT/n2_run.json 2> $OUT/n2_run.err || { echo "torchrun failed"; tail -20 $OUT/n2_run.err; exit 1; }
echo "torch.distributed.run N=2: $(( $(date +%s) - s )) s"
tail -1 $OUT/n2_run.json | cut -c1-600

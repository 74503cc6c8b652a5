#!/bin/bash
# round 4: the N > 1 line (the target list sharded over the ranks): its GPU tests at world 1 over RCCL, the
# driver's N = 2 command shape on the one-GPU box (both ranks on GPU 0, gloo), and rank 0's shard alone at N = 1
# for 2 / 4 / 8 ranks (what each rank's launches look like on its own GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04b}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_dist.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
s=$(date +%s)
timeout -k 10 500 python -u bench.py --gpus 2 --steps 50 --warmup 5 > $OUT/n2.json 2> $OUT/n2.err || { echo "n2 failed"; tail -30 $OUT/n2.err; exit 1; }
echo "N=2: $(( $(date +%s) - s )) s"
for n in 2 4 8; do
  timeout -k 10 300 python -u bench.py --shard 0/$n --steps 50 --warmup 5 > $OUT/shard0of$n.json 2> $OUT/shard0of$n.err || { echo "shard $n failed"; tail -30 $OUT/shard0of$n.err; exit 1; }
done
echo "shards ok"

# Flow rehearsal of the N>1 bench path on a 1-GPU box (2 ranks share GPU 0, gloo barriers). Not a scaling number.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rehearse
OVL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/rehearse/n2.json 2> gpurun_out/rehearse/n2.err; rc=$?
echo "rc=$rc"; tail -1 gpurun_out/rehearse/n2.json | cut -c1-700; tail -5 gpurun_out/rehearse/n2.err
exit $rc

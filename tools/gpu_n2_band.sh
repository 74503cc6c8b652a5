mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "rccl" > gpurun_out/pipe3.log 2>&1 || { tail -30 gpurun_out/pipe3.log; exit 1; }
tail -2 gpurun_out/pipe3.log
OVL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/n2b.json 2> gpurun_out/n2b.err || { tail -30 gpurun_out/n2b.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/n2b.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d.get('cfg5_band_sweep_sharded')))"

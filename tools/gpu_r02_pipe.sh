#!/bin/bash
# round 2: pipeline / multi-device / sharded tests, then a quick bench line (no extras)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r02_pipe.log 2>&1 || { echo "pipeline tests failed"; tail -40 gpurun_out/r02_pipe.log; exit 1; }
tail -3 gpurun_out/r02_pipe.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-extra --cpu-budget 4 \
  > gpurun_out/r02_bench_quick.json 2> gpurun_out/r02_bench_quick.err || { echo "bench failed"; tail -30 gpurun_out/r02_bench_quick.err; exit 1; }
cat gpurun_out/r02_bench_quick.json

#!/bin/bash
# round 2: pipeline tests with direct host stores, then the host-result path A/B (tools/pipe_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r02_pipe.log 2>&1 || { echo "pipeline tests failed"; tail -40 gpurun_out/r02_pipe.log; exit 1; }
tail -3 gpurun_out/r02_pipe.log
timeout -k 10 300 python -u tools/pipe_ab.py target > gpurun_out/r02_pipe_ab_target.json 2>&1 || { tail -30 gpurun_out/r02_pipe_ab_target.json; exit 1; }
cat gpurun_out/r02_pipe_ab_target.json
timeout -k 10 300 python -u tools/pipe_ab.py cfg4 > gpurun_out/r02_pipe_ab_cfg4.json 2>&1 || { tail -30 gpurun_out/r02_pipe_ab_cfg4.json; exit 1; }
cat gpurun_out/r02_pipe_ab_cfg4.json

# parity + pipeline GPU tests, then the per-call overhead probe (cfg2, target)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/q/pytest.log 2>&1 || { tail -40 gpurun_out/q/pytest.log; exit 1; }
tail -2 gpurun_out/q/pytest.log
timeout -k 10 200 python tools/step_overhead.py cfg2 2000 > gpurun_out/q/ovh_cfg2.json && timeout -k 10 200 python tools/step_overhead.py target 300 > gpurun_out/q/ovh_target.json && cat gpurun_out/q/ovh_*.json

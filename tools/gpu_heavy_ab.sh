# heavy tiles first: parity + pipeline tests, then kernel-only and step A/B at the target point and cfg3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/hv
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hv/pytest.log 2>&1 || { tail -30 gpurun_out/hv/pytest.log; exit 1; }
tail -1 gpurun_out/hv/pytest.log
timeout -k 10 300 python tools/heavy_first_ab.py target 5 20 > gpurun_out/hv/target.json && cat gpurun_out/hv/target.json && \
timeout -k 10 300 python tools/heavy_first_ab.py cfg3 3 10 > gpurun_out/hv/cfg3.json && cat gpurun_out/hv/cfg3.json

# pipeline + parity GPU tests, then the host-array entry points A/B (direct vs copy engine; 1 vs default copy threads)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/hp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/hp/pytest.log 2>&1 || { tail -40 gpurun_out/hp/pytest.log; exit 1; }
tail -2 gpurun_out/hp/pytest.log
timeout -k 10 300 python tools/host_paths_ab.py target 20 > gpurun_out/hp/target.json && cat gpurun_out/hp/target.json
OVL_HOST_THREADS=1 timeout -k 10 300 python tools/host_paths_ab.py target 20 > gpurun_out/hp/target_t1.json && cat gpurun_out/hp/target_t1.json

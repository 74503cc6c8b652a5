set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/uni
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/uni/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/uni/pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_rehearse_n2.sh

# packed polled expansion: the packed-transport tests only, verbose
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -k "packed" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pp/dbg.log 2>&1; grep -E "incomplete|passed|failed" gpurun_out/pp/dbg.log | head -20

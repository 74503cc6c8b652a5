set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05t6; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BANDS="-1 64 32 16 8 4" bash tools/gpu_r05_cfg5_pmc.sh r05cfg5c

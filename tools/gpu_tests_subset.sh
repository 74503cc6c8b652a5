#!/bin/bash
# a subset of the GPU tests on the box: bash tools/gpu_tests_subset.sh TAG test_file [test_file ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; shift
mkdir -p $OUT
FILES=""; for f in "$@"; do FILES="$FILES tests/$f"; done
timeout -k 10 900 python -u -m pytest $FILES -x -v --timeout 300 --timeout-method thread --durations=15 \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -60 $OUT/tests.log; exit 1; }
tail -25 $OUT/tests.log

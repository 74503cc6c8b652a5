#!/bin/bash
# progressive transport: its GPU tests, the pipeline and parity suites, then an interleaved A/B of the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prog
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread -k progressive \
  > $OUT/prog_tests.log 2>&1 || { echo "progressive tests failed"; tail -40 $OUT/prog_tests.log; exit 1; }
tail -4 $OUT/prog_tests.log
timeout -k 10 300 python -u tools/pack_ab.py target 5 20 > $OUT/ab_target.json 2> $OUT/ab_target.err \
  || { echo "ab failed"; tail -20 $OUT/ab_target.err; exit 1; }
cat $OUT/ab_target.json

#!/bin/bash
# round 4: the banded tests with the two-lane band kernel, then the band A/B (one vs two lanes per pair)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_banded.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/banded_tests.log 2>&1 || { echo "banded tests failed"; tail -40 $OUT/banded_tests.log; exit 1; }
tail -2 $OUT/banded_tests.log
timeout -k 10 400 python -u tools/band_ab.py 3 5 > $OUT/band_ab.json 2> $OUT/band_ab.err || { echo "band ab failed"; tail -30 $OUT/band_ab.err; exit 1; }
echo "band ab ok"
timeout -k 10 60 genome-assembly-using-overlap-graphs_amd/build/lane16_probe > $OUT/lane16_probe.txt 2>&1 || { echo "probe failed"; cat $OUT/lane16_probe.txt; exit 1; }
cat $OUT/lane16_probe.txt

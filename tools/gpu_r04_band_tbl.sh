#!/bin/bash
# round 4: band kernels, A/B of the previous build (build/ablate_oldband) against the new one: banded parity on the
# new build, then cfg5 band times of both in alternating
# processes (tools/band_ab.py, one lane and two lanes per pair)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04bt}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_banded.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "banded tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OLD="$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd/build/ablate_oldband/libovl.so"
for pass in 1 2; do
  for L in old new; do
    if [ $L = old ]; then LP="OVL_LIB_PATH=$OLD"; else LP=""; fi
    env $LP BAND_AB_BANDS=${BANDS:-8,16,32,48,64} timeout -k 10 300 python -u tools/band_ab.py 3 5 > $OUT/${L}_$pass.json 2>>$OUT/err.log || { echo "band ab failed $L"; tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/${L}_$pass.json'))
print('$L pass $pass', ' '.join(f\"{b}:{v['lane1']['median']}/{v['lane2']['median']}\" for b, v in d['ms'].items()))"
  done
done

#!/bin/bash
# A/B of the band kernels' body loop: eight rows per trip (default) against four (make -C
# genome-assembly-using-overlap-graphs_amd/csrc variant_lane V=unroll1 DEFS=-DOVL_BAND_UNROLL1), cfg5 bands
# 64 / 32 / 8 / 4, two passes each; the banded GPU tests first.
# usage: bash tools/gpu_band_unroll_ab.sh [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-unrollab}; mkdir -p $O; export TMPDIR=/tmp
V=genome-assembly-using-overlap-graphs_amd/build/ablate_unroll1/libovl.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_banded.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
ARGS="--config cfg5 --band-sweep=64,32,8,4 --sweep-steps 5 --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
for pass in 1 2; do
  timeout -k 10 300 python3 bench.py $ARGS > $O/u2_$pass.log 2>&1 || { tail -20 $O/u2_$pass.log; exit 1; }
  OVL_LIB_PATH=$V timeout -k 10 300 python3 bench.py $ARGS > $O/u1_$pass.log 2>&1 || { tail -20 $O/u1_$pass.log; exit 1; }
done
for f in u2_1 u1_1 u2_2 u1_2; do python3 -c "
import json
for l in open('$O/$f.log'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); print('$f', [(p['band'], round(p['kernel_ms'],3)) for p in d['band_sweep']['points']])"; done
echo ok

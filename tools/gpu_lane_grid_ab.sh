#!/bin/bash
# A/B of the lane kernels' grid, cfg5 points: full DP int32 (OVL_LANE_FORM=3), bands 64 / 32 / 8.  Round 5 ran it
# when resident slots looping over the tiles was the default and "all" a variant; now every tile launched is the
# default and the slots grid the variant: make -C genome-assembly-using-overlap-graphs_amd/csrc variant_lane
# V=gridall DEFS=-DOVL_LANE_GRID_SLOTS (the labels def/all then swap).
# usage: bash tools/gpu_lane_grid_ab.sh [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-gridab}; mkdir -p $O; export TMPDIR=/tmp
V=genome-assembly-using-overlap-graphs_amd/build/ablate_gridall/libovl.so
ARGS="--config cfg5 --band-sweep=-1,64,32,8 --sweep-steps 5 --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
for pass in 1 2; do
  OVL_LANE_FORM=3 timeout -k 10 300 python3 bench.py $ARGS > $O/def$pass.log 2>&1 || { tail -20 $O/def$pass.log; exit 1; }
  OVL_LANE_FORM=3 OVL_LIB_PATH=$V timeout -k 10 300 python3 bench.py $ARGS > $O/all$pass.log 2>&1 || { tail -20 $O/all$pass.log; exit 1; }
done
for f in def1 all1 def2 all2; do python3 -c "
import json
for l in open('$O/$f.log'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); print('$f', [(p['band'], p.get('kernel'), round(p['kernel_ms'],3)) for p in d['band_sweep']['points']])"; done
echo ok
# the h2 kernel's hand-off, HBM against LDS (round 5: LDS the default, HBM the variant; now HBM is the default and
# the variant is make variant_lane V=h2hbm DEFS=-DOVL_H2_LDS, labels swapped): its lane tests, then cfg5's full DP
V2=genome-assembly-using-overlap-graphs_amd/build/ablate_h2hbm/libovl.so
if [ -f $V2 ]; then
  OVL_LIB_PATH=$V2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dp_lane.py -x -q -k "h2" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/hbm_tests.log 2>&1 || { tail -20 $O/hbm_tests.log; exit 1; }
  tail -1 $O/hbm_tests.log
  A2="--config cfg5 --band-sweep=-1 --sweep-steps 5 --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
  for pass in 1 2; do
    timeout -k 10 300 python3 bench.py $A2 > $O/h2lds$pass.log 2>&1 || { tail -20 $O/h2lds$pass.log; exit 1; }
    OVL_LIB_PATH=$V2 timeout -k 10 300 python3 bench.py $A2 > $O/h2hbm$pass.log 2>&1 || { tail -20 $O/h2hbm$pass.log; exit 1; }
  done
  for f in h2lds1 h2hbm1 h2lds2 h2hbm2; do python3 -c "
import json
for l in open('$O/$f.log'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); print('$f', [(p['band'], p.get('kernel'), round(p['kernel_ms'],3)) for p in d['band_sweep']['points']])"; done
fi
echo done2

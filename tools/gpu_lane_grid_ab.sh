#!/bin/bash
# A/B of the lane kernels' grid: resident slots looping over the tiles (default build) against a tile per wavefront
# (build/ablate_gridall, -DOVL_LANE_GRID_ALL), cfg5 points: full DP int32 (OVL_LANE_FORM=3), bands 64 / 32 / 8.
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

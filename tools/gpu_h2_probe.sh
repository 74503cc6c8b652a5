#!/bin/bash
# Round-5 probe of dp_lane_h2_kernel (two pairs per lane, packed f16): the lane tests, then cfg5's full DP point
# under rocprofv3 (default build), then the int32 lane kernel (OVL_LANE_FORM=3) and the default again; with
# build/ablate_persist (make variant_lane V=persist DEFS=-DOVL_LANE_GRID_SLOTS) the resident-slots grid too.
# usage: bash tools/gpu_h2_probe.sh [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-h2a}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dp_lane.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
ARGS="--config cfg5 --band-sweep=-1 --sweep-steps 5 --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py $ARGS > $O/b.log 2>&1 || { tail -30 $O/b.log; exit 1; }
OVL_LANE_FORM=3 timeout -k 10 300 python3 bench.py $ARGS > $O/b3.log 2>&1 || { tail -30 $O/b3.log; exit 1; }
timeout -k 10 300 python3 bench.py $ARGS > $O/b7.log 2>&1 || { tail -30 $O/b7.log; exit 1; }
if [ -f genome-assembly-using-overlap-graphs_amd/build/ablate_persist/libovl.so ]; then
  OVL_LIB_PATH=genome-assembly-using-overlap-graphs_amd/build/ablate_persist/libovl.so timeout -k 10 300 python3 bench.py $ARGS > $O/bp.log 2>&1 || { tail -30 $O/bp.log; exit 1; }
fi
for f in b3 b7 bp; do [ -f $O/$f.log ] || continue; python3 -c "
import json,sys
for l in open('$O/$f.log'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); p=d['band_sweep']['points'][0]; print('$f', p.get('kernel'), p.get('kernel_ms'), p.get('ms_per_step'))"; done
echo ok

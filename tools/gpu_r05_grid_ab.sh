#!/bin/bash
# round 5: uniform_kernel grid cap (blocks of 256 per CU, build macro OVL_BLOCKS_PER_CU) against the per-rank steps
# (tools/shard_step_ab.py, N = 1 and 8), each build in its own process through OVL_LIB_PATH, two passes
# usage: bash tools/gpu_r05_grid_ab.sh [tag]    (builds: make -C genome-assembly-using-overlap-graphs_amd/csrc variant ...)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r05grid}
mkdir -p $OUT
B=genome-assembly-using-overlap-graphs_amd/build
for pass in ${PASSES:-1 2}; do
  for v in ${VARIANTS:-default bpc8 bpc16 bpc64}; do
    if [ $v = default ]; then LIB=$B/libovl.so; else LIB=$B/ablate_$v/libovl.so; fi
    OVL_LIB_PATH=$LIB SHARD_AB_NS=1,8 timeout -k 10 200 python3 -u tools/shard_step_ab.py 3 30 > $OUT/${v}_$pass.json \
      2> $OUT/${v}_$pass.err || { echo "$v failed"; tail -20 $OUT/${v}_$pass.err; exit 1; }
    echo "$v pass $pass ok"
  done
done
echo all ok

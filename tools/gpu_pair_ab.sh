#!/bin/bash
# round 3: shift-pair sweep A/B (default build = keys_s2 / keys_t2, build/ablate_nopair = one shift per s shift):
# parity subset on the default build, then target point and cfg3, interleaved passes.  Build the variant first:
#   make -C genome-assembly-using-overlap-graphs_amd/csrc variant V=nopair DEFS="-DOVL_SHIFT_PAIR=0"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_lib_ab.sh ${1:-r03h_pair} nopair 3 default || exit 1
BENCH_ARGS="--config cfg3" bash tools/gpu_lib_ab.sh ${1:-r03h_pair}_cfg3 nopair 2 none || exit 1

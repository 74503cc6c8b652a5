#!/bin/bash
# round 4: software prefetch of the packed source in the AVX-512 expansion (ovl_expand.h OVL_EXPAND_PF /
# OVL_EXPAND_PF_PART), the expansion probe built per setting, bound to the GPU's NUMA node, two interleaved rounds.
# Record of a rejected experiment: no distance helped (profiles/r04_expand_prefetch_ab.txt), so the two macros
# were taken out of ovl_expand.h again; to rerun, put the prefetch back and build each probe with -D<macro>=<v>.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04pf}
mkdir -p $OUT
B=genome-assembly-using-overlap-graphs_amd/build/expand_probe
for round in 1 2; do
  for v in pf0 pf256 pf512 pf1k pf2k pf4k part; do
    timeout -k 10 120 ${B}_$v 40 -2 > $OUT/${v}_$round.txt 2>&1 || { echo "$v failed"; cat $OUT/${v}_$round.txt; exit 1; }
    echo "== $v round $round"; grep -E "node|kernel-written -> pinned coherent dst \(the step\)|coherent src \(warm\)" $OUT/${v}_$round.txt
  done
done

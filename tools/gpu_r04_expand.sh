#!/bin/bash
# round 4: the expansion probe unbound and bound to the GPU's NUMA node (and the other node)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04x}
mkdir -p $OUT
# the visible GPU's node from its PCI address (the probe's "-2"); the first /sys/class/drm card, which this script
# read before, can be another GPU of the host on another node
NODE=$(genome-assembly-using-overlap-graphs_amd/build/expand_probe 0 -2 | sed -n 's/^gpu .* node \(-\?[0-9]*\)$/\1/p')
echo "gpu node $NODE"
B=genome-assembly-using-overlap-graphs_amd/build/expand_probe
timeout -k 10 120 $B 30 -1 > $OUT/unbound.txt 2>&1 || { echo "unbound failed"; cat $OUT/unbound.txt; exit 1; }
cat $OUT/unbound.txt
if [ "$NODE" -ge 0 ]; then
  timeout -k 10 120 $B 30 $NODE > $OUT/node$NODE.txt 2>&1 || { echo "bound failed"; cat $OUT/node$NODE.txt; exit 1; }
  cat $OUT/node$NODE.txt
  OTHER=$(( NODE == 0 ? 1 : 0 ))
  timeout -k 10 120 $B 30 $OTHER > $OUT/node$OTHER.txt 2>&1 || { echo "other failed"; cat $OUT/node$OTHER.txt; exit 1; }
  cat $OUT/node$OTHER.txt
fi

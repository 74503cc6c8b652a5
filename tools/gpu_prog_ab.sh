#!/bin/bash
# progressive transport A/B (tools/pack_ab.py, interleaved engines) at the target point and cfg3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prog
mkdir -p $OUT
for cfg in target cfg3; do
  timeout -k 10 300 python -u tools/pack_ab.py $cfg 7 20 > $OUT/ab2_$cfg.json 2> $OUT/ab2_$cfg.err \
    || { echo "ab $cfg failed"; tail -20 $OUT/ab2_$cfg.err; exit 1; }
  cat $OUT/ab2_$cfg.json
done

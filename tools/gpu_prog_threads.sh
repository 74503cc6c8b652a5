#!/bin/bash
# host pool size with the progressive transport: alternating processes of 12 and 15 threads (tools/pack_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prog_threads
mkdir -p $OUT
for i in 1 2 3; do
  for t in 12 15; do
    OVL_HOST_THREADS=$t timeout -k 10 200 python -u tools/pack_ab.py target 5 20 > $OUT/t${t}_$i.json 2> $OUT/t${t}_$i.err \
      || { echo "run t=$t failed"; tail -20 $OUT/t${t}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/t${t}_$i.json')); print($t, $i, d['progressive']['pinned']['median_ms'], d['packed_adaptive']['pinned']['median_ms'])"
  done
done

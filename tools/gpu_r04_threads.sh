#!/bin/bash
# round 4: host pool threads for the N = 1 step (12 = the rule's cap, against 14 and 15 of the box's 16-CPU share),
# alternating processes (the pool is sized once per process)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04th}
mkdir -p $OUT
for i in 1 2 3; do
  for t in 12 14 15; do
    OVL_POOL_THREADS=$t timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra > $OUT/t$t.$i.json 2> $OUT/t$t.$i.err || { echo "t$t $i failed"; tail -20 $OUT/t$t.$i.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/t$t.$i.json') if l.startswith('{')][-1]); print('threads $t', $i, round(d['ms_per_step'],4))"
  done
done

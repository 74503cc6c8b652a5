#!/bin/bash
# round 4: the N = 1 step with the process on its GPU's NUMA node (the default since) against --no-numa-bind, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04n}
mkdir -p $OUT
for i in 1 2 3; do
  for mode in default bind; do
    extra="--no-numa-bind"; [ $mode = bind ] && extra=""
    timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra $extra > $OUT/$mode.$i.json 2> $OUT/$mode.$i.err || { echo "$mode $i failed"; tail -20 $OUT/$mode.$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$mode.$i.json') if l.startswith('{')][-1]); print('$mode', $i, round(d['ms_per_step'],4), d.get('rank0_numa_node', d.get('config',{}).get('rank0_numa_node')))"
  done
done

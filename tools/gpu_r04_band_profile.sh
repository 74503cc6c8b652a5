#!/bin/bash
# round 4 band sweep (BASELINE configs[4], cfg5) on the final tree: rocprofv3 kernel trace + stats of the bench's
# band sweep, one launch pair (seed + band kernel) per step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-r04band}"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg5 --band-sweep 4,8,16,24,32,48,64,-1 --sweep-steps 5 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > "$OUT/kt.log" 2>&1 || { echo "failed"; tail -20 "$OUT/kt.log"; exit 1; }
grep '^{"metric"' "$OUT/kt.log" | python3 -c "
import json, sys; d = json.loads(sys.stdin.read())
for p in d['band_sweep']['points']: print(p['band'], p['kernel'], round(p['ms_per_step'], 3), round(p.get('kernel_ms', 0), 3))"

# A/B of the uniform kernel launch mode (OVL_SPLIT=0 normal, 1 latency mode; 2 = same as 1) on cfg2 and target, kernel-only timing from bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-splitab}"
mkdir -p "$OUT"
for cfg in cfg2 target; do
  for s in 0 1 2; do
    OVL_SPLIT=$s timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 10 --no-cpu-baseline --no-extra > "$OUT/${cfg}_s$s.json" 2>>"$OUT/err.log" || { echo "failed $cfg $s"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/${cfg}_s$s.json').read().strip().splitlines()[-1]); print('$cfg split=$s', round(d['value']/1e9,3), 'Gpairs/s kernel_ms', round(d['roofline']['kernel_ms']*1000,2), 'us')"
  done
done

# A/B of the ungapped grid cap (OVL_BLOCKS_PER_CU) on cfg2 and target, kernel-only timing from bench.
set -u
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-gridab}"
mkdir -p "$OUT"
for cfg in cfg2 target; do
  for b in ${2:-4 8 16 32 64}; do
    OVL_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 10 --no-cpu-baseline --no-extra > "$OUT/${cfg}_b$b.json" 2>>"$OUT/err.log" || { echo "failed $cfg $b"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/${cfg}_b$b.json').read().strip().splitlines()[-1]); print('$cfg blocks/CU=$b', round(d['value']/1e9,3), 'Gpairs/s kernel', round(d['roofline']['kernel_ms']*1000,2), 'us')"
  done
done

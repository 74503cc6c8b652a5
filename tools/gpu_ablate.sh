# Kernel-time ablation on cfg2/target: full build vs no sweep (loads kept) vs no row loads (sweep kept). Timing only.
set -u
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-ablate}"; mkdir -p "$OUT"
for v in full SWEEP LOADS; do
  if [ $v = full ]; then L="$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd/build/libovl.so"; else L="$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd/build/ablate_$v/libovl.so"; fi
  for cfg in cfg2 target; do
    OVL_LIB_PATH=$L timeout -k 10 200 python bench.py --config $cfg --steps 200 --warmup 10 --no-cpu-baseline --no-extra > "$OUT/${cfg}_$v.json" 2>>"$OUT/err.log" || { echo "failed $v $cfg"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${cfg}_$v.json').read().strip().splitlines()[-1]); print('$v $cfg kernel_us', round(d['kernel_only_roofline']['kernel_ms']*1000,2))"
  done
done

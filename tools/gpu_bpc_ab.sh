#!/bin/bash
# kernel-only time of the target list vs the uniform kernel's grid cap (OVL_BLOCKS_PER_CU), two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-bpc}
mkdir -p $OUT
for pass in 1 2; do
  for b in 8 16 32 64; do
    OVL_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extra > $OUT/b${b}_$pass.json 2>>$OUT/err.log || { echo "failed $b"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b${b}_$pass.json').read().strip().splitlines()[-1]); print('bpc $b pass $pass kernel_us', round(d['kernel_only_roofline']['kernel_ms']*1000,2), 'step_ms', round(d['ms_per_step'],4))"
  done
done

#!/bin/bash
# kernel-only and step time of the default bench workload under environment settings, interleaved passes:
#   bash tools/gpu_env_ab.sh TAG PASSES "A=1" "A=0 B=2" ...   ("-" = no setting)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; PASSES=$2; shift 2
mkdir -p $OUT
for pass in $(seq 1 $PASSES); do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    envs=""; [ "$setting" != "-" ] && envs="$setting"
    env $envs timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extra > $OUT/s${i}_$pass.json 2>>$OUT/err.log || { echo "failed $setting"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/s${i}_$pass.json').read().strip().splitlines()[-1]); print('[$setting] pass $pass kernel_us', round(d['kernel_only_roofline']['kernel_ms']*1000,2), 'step_ms', round(d['ms_per_step'],4), 'in-step packed us', round(d['roofline']['launch_ms']*1000,2))"
  done
done

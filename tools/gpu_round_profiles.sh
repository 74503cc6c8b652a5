# Round-end evidence on the GPU box: bench + rocprof stats + FETCH/WRITE passes + VALU PMC passes for
# cfg2 and the target point, the default bench line, and the cfg5 band sweep.
# usage: bash tools/gpu_round_profiles.sh <round-tag>
set -u
R=${1:-r01}
cd "$GRAFT_REPO_ROOT"
for cfg in cfg2 target; do
  bash tools/gpu_profile.sh "${R}_prof_$cfg" $cfg || exit 1
  bash tools/gpu_pmc.sh "${R}_valu_$cfg" $cfg "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_INSTS_SALU" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD" || exit 1
done
mkdir -p gpurun_out/$R
timeout -k 10 400 python bench.py > gpurun_out/$R/bench_default.json 2> gpurun_out/$R/bench_default.err || exit 1
timeout -k 10 400 python bench.py --config cfg5 --steps 20 --warmup 2 --no-extra --no-cpu-baseline --band-sweep 8,16,32,64,-1 > gpurun_out/$R/cfg5_sweep.json 2> gpurun_out/$R/cfg5_sweep.err || exit 1
echo done

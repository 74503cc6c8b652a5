# Round evidence for the gapped kernels: kernel-trace stats of the cfg5 band sweep and the cfg2 extras,
# then PMC passes (VALU issue, HBM traffic) for dp_lane_kernel (cfg5 full DP, indel -2) and
# band_lane_kernel (cfg5 band 8).  usage: bash tools/gpu_profiles_lane.sh <tag>
set -u
T=${1:-r01_lane}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_profile_extras.sh "$T" || exit 1
for spec in "full|--config cfg5 --steps 5 --warmup 1 --indel -2 --band -1" "band8|--config cfg5 --steps 5 --warmup 1 --indel -2 --band 8"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-extra > gpurun_out/$T/bench_$name.json 2> gpurun_out/$T/bench_$name.err || exit 1
  bash tools/gpu_pmc_args.sh "$T/pmc_$name" "$args" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "FETCH_SIZE" "WRITE_SIZE" || exit 1
done
echo done

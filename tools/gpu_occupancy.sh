# Occupancy / LDS PMC passes for the headline kernel (uniform_kernel) at cfg2 and the target point.
# usage: bash tools/gpu_occupancy.sh <tag>
set -u
T=${1:-r01_occ}
cd "$GRAFT_REPO_ROOT"
for cfg in cfg2 target; do
  bash tools/gpu_pmc.sh "$T/$cfg" $cfg "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" || exit 1
done
echo done

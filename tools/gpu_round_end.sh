# Round-end pass: smoke + pytest -m gpu + short bench, then rocprof/PMC profiles and occupancy passes.
# usage: bash tools/gpu_round_end.sh <round-tag>
set -u
R=${1:-r01}
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh && bash tools/gpu_round_profiles.sh "$R" && bash tools/gpu_occupancy.sh "${R}_occ"

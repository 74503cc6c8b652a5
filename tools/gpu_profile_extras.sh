# rocprofv3 kernel-trace/stats for the non-metric kernels: cfg5 band sweep (seed + band_diag_kernel / dp_fast_kernel),
# device candidate enumeration + local alignment (bench extras at cfg2).  usage: bash tools/gpu_profile_extras.sh <tag>
set -u
TAG=${1:-extras}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/band" -o band --output-format csv -- python3 "$B" --config cfg5 --steps 5 --warmup 1 --no-extra --no-cpu-baseline --band-sweep 4,8,16,24,32,48,64,-1 > "$OUT/band.log" 2>&1 || { echo "band failed"; tail -20 "$OUT/band.log"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/extras" -o extras --output-format csv -- python3 "$B" --config cfg2 --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/extras.log" 2>&1 || { echo "extras failed"; tail -20 "$OUT/extras.log"; exit 1; }
cut -c1-160 "$OUT/band/band_kernel_stats.csv"; cut -c1-160 "$OUT/extras/extras_kernel_stats.csv"

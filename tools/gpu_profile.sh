# Bench + rocprofv3 kernel-trace/stats + separate FETCH_SIZE / WRITE_SIZE passes (dominant kernel) on the GPU box.
# usage: bash tools/gpu_profile.sh <tag> [config] [kernel-regex]
set -u
TAG=${1:-r01}
CFG=${2:-cfg2}
KRX=${3:-uniform_kernel}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
echo "== bench $CFG"
timeout -k 10 400 python "$B" --config "$CFG" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json" | cut -c1-600
echo "== kernel trace + stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 "$B" --config "$CFG" --steps 200 --warmup 10 --no-cpu-baseline --no-extra > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$OUT/kt.log"; exit 1; }
cat "$OUT/kt/kt_kernel_stats.csv"
echo "== pmc FETCH_SIZE"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --kernel-include-regex "$KRX" -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$B" --config "$CFG" --steps 30 --warmup 2 --no-cpu-baseline --no-extra > "$OUT/fetch.log" 2>&1 || { echo "fetch failed"; tail -20 "$OUT/fetch.log"; exit 1; }
echo "== pmc WRITE_SIZE"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --kernel-include-regex "$KRX" -d "$OUT/write" -o write --output-format csv -- python3 "$B" --config "$CFG" --steps 30 --warmup 2 --no-cpu-baseline --no-extra > "$OUT/write.log" 2>&1 || { echo "write failed"; tail -20 "$OUT/write.log"; exit 1; }
echo done

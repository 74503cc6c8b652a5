# GPU parity suite + bench (+ optional rocprof kernel trace). usage: bash tools/gpu_quick.sh <tag> [kt]
set -u
TAG=${1:-dev}
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest gpu"
timeout -k 10 900 python -m pytest tests/ -q -m gpu --maxfail=5 -p no:cacheprovider --durations=8 > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" "$OUT/pytest_gpu.log" | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== bench"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json"
if [ "${2:-}" = "kt" ]; then
  echo "== kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 5 --no-cpu-baseline > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$OUT/kt.log"; exit 1; }
  cat "$OUT/kt/kt_kernel_stats.csv"
fi
exit $rc

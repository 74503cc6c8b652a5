# PMC counter passes (each its own rocprofv3 run, kernel-trace only) on one bench invocation.
# usage: bash tools/gpu_pmc_args.sh <tag> "<bench args>" "<counters pass 1>" "<counters pass 2>" ...
set -u
TAG=$1; ARGS=$2; shift 2
cd "$GRAFT_REPO_ROOT"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for CTRS in "$@"; do
  i=$((i+1))
  echo "== pass $i: $CTRS"
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace -T -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS --no-cpu-baseline --no-extra > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
echo done

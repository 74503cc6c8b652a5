#!/bin/bash
# round 2 profiles of the default bench command's workload (target point): GPU tests, kernel trace + stats,
# FETCH_SIZE / WRITE_SIZE passes (separate runs), and the processes left after bench exits.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/r02prof"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
  || { echo "gpu tests failed"; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
echo "== kernel trace + stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- python3 "$B" --steps 20 --warmup 5 --no-cpu-baseline --no-extra > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$OUT/kt.log"; exit 1; }
KT=$(find "$OUT/kt" -name "kt_kernel_trace.csv" | head -1)
python3 tools/kt_phases.py "$KT" uniform_kernel 5 20 "$OUT/phases.json"
echo "== pmc FETCH_SIZE"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --kernel-include-regex uniform_kernel -d "$OUT/fetch" -o fetch --output-format csv -- python3 "$B" --steps 20 --warmup 5 --no-cpu-baseline --no-extra > "$OUT/fetch.log" 2>&1 || { echo "fetch failed"; tail -20 "$OUT/fetch.log"; exit 1; }
echo "== pmc WRITE_SIZE"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --kernel-include-regex uniform_kernel -d "$OUT/write" -o write --output-format csv -- python3 "$B" --steps 20 --warmup 5 --no-cpu-baseline --no-extra > "$OUT/write.log" 2>&1 || { echo "write failed"; tail -20 "$OUT/write.log"; exit 1; }
echo "== processes after bench"
timeout -k 10 300 python3 "$B" --steps 20 --warmup 5 --no-extra --cpu-budget 2 > "$OUT/bench_ps.json" 2>&1; echo "bench rc=$?"
sleep 1
ps -u "$(id -u)" -o pid,ppid,stat,etime,cmd > "$OUT/ps_after.txt"; cat "$OUT/ps_after.txt"
echo done

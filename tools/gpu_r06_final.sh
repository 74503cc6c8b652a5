#!/bin/bash
# Round-6 final tier on one box: the GPU tests, smoke, the default bench line (N = 1), the N = 2 launcher
# rehearsal (both ranks on the one GPU), and a rocprofv3 kernel trace + stats of a short default bench run. Each step under its own time limit; the first failure ends the run.
# usage: bash tools/gpu_r06_final.sh [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="gpurun_out/${1:-r06final}"
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python3 -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
echo "== smoke"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -30 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
echo "== bench N = 1"
timeout -k 10 900 python3 -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$OUT/bench.log"; exit 1; }
grep '^{"metric"' "$OUT/bench.log" > "$OUT/bench.json"
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', d['roofline']['frac'])
e = d.get('end_to_end') or {}; print('end_to_end', {k: v for k, v in e.items() if 'remove' in k})"
echo "== bench N = 2 rehearsal (two ranks on one GPU)"
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_n2.log" 2>&1 \
  || { echo "bench N=2 failed"; tail -30 "$OUT/bench_n2.log"; exit 1; }
grep '^{"metric"' "$OUT/bench_n2.log" > "$OUT/bench_n2.json"
echo "== rocprofv3 kernel trace + stats of the default bench (short)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra > "$OUT/prof.log" 2>&1 \
  || { echo "profile failed"; tail -30 "$OUT/prof.log"; exit 1; }
echo all ok

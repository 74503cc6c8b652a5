#!/bin/bash
# Round 6: the resident scoring grid on the box -- its GPU tests, then per-rank steps (tools/shard_step_ab.py) of the
# resident grid at 1 / 2 / 4 blocks per CU against the launch pipeline.  Output under gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r06res}
mkdir -p "$out"
timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread \
    > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
SHARD_AB_SETTINGS="${SETTINGS:-resident2=OVL_RESIDENT:1x2;resident1=OVL_RESIDENT:1x1;resident4=OVL_RESIDENT:1x4;pipeline=OVL_RESIDENT:0}" \
    timeout -k 10 400 python -u tools/shard_step_ab.py "${ROUNDS:-3}" "${REPS:-30}" > "$out/shards.json" 2> "$out/shards.err" \
    || { echo "shard_step_ab failed"; tail -20 "$out/shards.err"; exit 1; }
python - "$out/shards.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
for r in d["results"]:
    print(f'{r["setting"]:>10} N={r["ranks"]} shard={r["shard_pairs"]:>8} median {r["median_ms"]:.4f} ms '
          f'(min {r["min_ms"]:.4f}, max {r["max_ms"]:.4f})')
EOF

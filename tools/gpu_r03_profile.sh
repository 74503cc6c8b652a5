#!/bin/bash
# Round-3 profiles of the default bench workload, the headline command without extras:
#   kernel trace + stats of every kernel (the step's uniform_kernel<W, 0, false, 2> packed chunks and <.., 1>
#   direct chunk, and the HBM-output <.., 0> that kernel_only_roofline times), then PMC passes, each in its
#   own run, over every uniform_kernel instantiation: FETCH_SIZE, WRITE_SIZE, SQ instruction counts and clock,
#   occupancy, LDS.
# usage: bash tools/gpu_r03_profile.sh [config] [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
CFG=${1:-target}
TAG=${2:-r03prof}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
ARGS="--config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-extra"
echo "== kernel trace + stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 "$B" $ARGS > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$OUT/kt.log"; exit 1; }
KRE="uniform_kernel"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  echo "== pmc pass $i: $CTRS"
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace --kernel-include-regex "$KRE" -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$B" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
echo done

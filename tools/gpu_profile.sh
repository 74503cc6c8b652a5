#!/bin/bash
# Round-4 profiles of the default bench workload (or a rank's shard: SHARD=0/8): kernel trace + stats, then PMC
# passes over every uniform_kernel instantiation, each in its own run:
#   FETCH_SIZE; WRITE_SIZE; VALU/SALU instruction counts, waves and clock; wave-cycle breakdown (resident,
#   parked on s_waitcnt, issue-stalled, issuing) -- the in-step kernels' stores go over the host link, so
#   SQ_WAIT_ANY against SQ_WAVE_CYCLES names how long their waves sit waiting for them; LDS instructions, bank
#   conflict and LDS-array cycles (round 6: the in-step kernel that stages rows in LDS)
# usage: bash tools/gpu_profile.sh [config] [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
CFG=${1:-target}
TAG=${2:-prof}
OUT="$GRAFT_REPO_ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
ARGS="--config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-extra"
[ -n "$SHARD" ] && ARGS="$ARGS --shard $SHARD"
echo "== kernel trace + stats ($ARGS)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 "$B" $ARGS > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$OUT/kt.log"; exit 1; }
KRE="uniform_kernel"
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc pass $i: $CTRS"
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace --kernel-include-regex "$KRE" -d "$OUT/p$i" -o p$i --output-format csv -- python3 "$B" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
done
echo done

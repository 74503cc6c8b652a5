#!/bin/bash
# Round-5 PMC of BASELINE configs[4] (cfg5): every point of the bench's band sweep -- the full reference DP (band -1,
# dp_lane_kernel), band 64 (band_lane2_kernel) and 4..32 (band_lane_kernel) -- one bench process per band and pass:
#   p1 instruction mix (VALU, SALU, LDS) + waves + clock; p2 wave-cycle breakdown + clock;
#   p3 LDS array cycles and bank-conflict cycles; p4 FETCH_SIZE
# usage: BANDS="-1 64 32 16 8 4" bash tools/gpu_r05_cfg5_pmc.sh [tag]      summary: python3 tools/cfg5_pmc_summary.py gpurun_out/<tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/${1:-r05cfg5}"
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py"
KRE="dp_lane|band_lane"
for BAND in ${BANDS:--1 64 32 16 8 4}; do
  ARGS="--config cfg5 --band-sweep=$BAND --sweep-steps 3 --steps 3 --warmup 1 --no-cpu-baseline --no-extra"
  D="$OUT/b$BAND"
  mkdir -p "$D"
  echo "== band $BAND kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$D/kt" -o kt --output-format csv -- python3 "$B" $ARGS > "$D/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$D/kt.log"; exit 1; }
  i=0
  for CTRS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
              "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
              "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" \
              "FETCH_SIZE"; do
    i=$((i+1))
    echo "== band $BAND pmc pass $i: $CTRS"
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $CTRS --kernel-trace --kernel-include-regex "$KRE" -d "$D/p$i" -o p$i --output-format csv -- python3 "$B" $ARGS > "$D/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$D/p$i.log"; exit 1; }
  done
done
echo done

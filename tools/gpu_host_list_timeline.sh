#!/bin/bash
# kernel trace of host-pair-list calls (tools/host_list_timeline.py), OVL_TRACE_PIPE host marks beside it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tl}
mkdir -p $OUT
OVL_TRACE_PIPE=1 timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/prof -o tl -- python3 tools/host_list_timeline.py target 10 \
  > $OUT/out.txt 2> $OUT/trace.txt || { echo "timeline failed"; tail -20 $OUT/trace.txt; exit 1; }
cat $OUT/out.txt
find $OUT/prof -name "*kernel_trace.csv" | head -3

#!/bin/bash
# ovl_set_reads: timeline (kernels + copies) and host marks, packed vs raw upload
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sr}
mkdir -p $OUT
OVL_TRACE_PIPE=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof -o sr -- \
  python3 tools/set_reads_timeline.py target 10 > $OUT/out.txt 2> $OUT/trace.txt || { echo "failed"; tail -20 $OUT/trace.txt; exit 1; }
cat $OUT/out.txt
OVL_TRACE_PIPE=1 timeout -k 10 240 python3 tools/set_reads_timeline.py target 30 > $OUT/out2.txt 2> $OUT/trace2.txt \
  || { echo "failed"; exit 1; }
cat $OUT/out2.txt

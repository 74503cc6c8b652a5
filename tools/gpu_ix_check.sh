#!/bin/bash
# compact pair-list tests (in-place IX and decode paths), the host-list timeline and the probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ix}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_compact_pairs.py -x -v --timeout 200 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OVL_TRACE_PIPE=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/prof -o tl -- python3 tools/host_list_timeline.py target 10 \
  > $OUT/tl_out.txt 2> $OUT/tl_trace.txt || { echo "timeline failed"; tail -20 $OUT/tl_trace.txt; exit 1; }
cat $OUT/tl_out.txt
for r in 1 2; do
  OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/host_list_probe.py target >> $OUT/probe.txt 2>> $OUT/probe_trace.txt \
    || { echo "probe failed"; exit 1; }
done
cat $OUT/probe.txt

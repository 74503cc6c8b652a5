#!/bin/bash
# read-upload forms (2-bit packed / raw), compact pair lists, the one-shot ABI tests, then the probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-rd}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact_pairs.py tests/test_gpu_c_abi.py \
  -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/host_list_probe.py target > $OUT/probe.txt 2> $OUT/probe_trace.txt \
  || { echo "probe failed"; exit 1; }
cat $OUT/probe.txt
grep -B3 "== set_reads above" $OUT/probe_trace.txt | head -4

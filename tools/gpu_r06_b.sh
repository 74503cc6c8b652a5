#!/bin/bash
# Round 6: GPU tests of the resident grid, device workers and device-count rule; the traced resident probe; the
# single-process N-slot probe.  Output under gpurun_out/$1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/${1:-r06b}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_pipeline.py tests/test_gpu_reads_resident.py \
    -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
OVL_TRACE_PIPE=1 timeout -k 10 300 python -u tools/resident_probe.py "${FORMS:-1x2x1x4,1x1x1x4}" 30 > "$out/probe.json" 2> "$out/probe.err" \
    || { echo "probe failed"; tail -5 "$out/probe.err"; exit 1; }
timeout -k 10 300 python -u tools/multidev_probe.py 30 > "$out/multidev.json" 2> "$out/multidev.err" \
    || { echo "multidev failed"; tail -5 "$out/multidev.err"; exit 1; }
echo ok

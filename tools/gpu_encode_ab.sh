#!/bin/bash
# compact pair-list tests, then the host-list probe with the scalar and the vector encoding (pipeline traces)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-enc}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact_pairs.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for isa in scalar "" scalar ""; do
  OVL_ENCODE_ISA=$isa OVL_TRACE_PIPE=1 timeout -k 10 200 python -u tools/host_list_probe.py target \
    >> $OUT/out_${isa:-vec}.txt 2>> $OUT/trace_${isa:-vec}.txt || { echo "probe failed"; exit 1; }
done
cat $OUT/out_scalar.txt $OUT/out_vec.txt

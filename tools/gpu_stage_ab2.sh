#!/bin/bash
# packed-chunk staging variants (OVL_PACK_STAGE 0 link stores / 1 copy kernel / 2 copy engine / 3 copy kernel at
# high priority), interleaved, fixed 18 % direct share and adaptive; plus the pipeline tests under each variant
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-stage2}
mkdir -p $OUT
for st in 2 3; do
  OVL_PACK_STAGE=$st timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread -k "packed or step_transport or heavy" > $OUT/tests_$st.log 2>&1 || { echo "tests $st failed"; tail -30 $OUT/tests_$st.log; exit 1; }
  tail -1 $OUT/tests_$st.log
done
export PACK_AB_SETTINGS="link=OVL_PACK_STAGE:0;kernel=OVL_PACK_STAGE:1;sdma=OVL_PACK_STAGE:2;prio=OVL_PACK_STAGE:3;link18=OVL_PACK_STAGE:0,OVL_PACK_DIRECT_PCT:18;sdma18=OVL_PACK_STAGE:2,OVL_PACK_DIRECT_PCT:18;prio18=OVL_PACK_STAGE:3,OVL_PACK_DIRECT_PCT:18;prio0=OVL_PACK_STAGE:3,OVL_PACK_DIRECT_PCT:0;sdma0=OVL_PACK_STAGE:2,OVL_PACK_DIRECT_PCT:0"
timeout -k 10 400 python -u tools/pack_ab.py target 5 20 > $OUT/ab_target.json 2> $OUT/ab_target.err || { echo "ab failed"; tail -20 $OUT/ab_target.err; exit 1; }
cat $OUT/ab_target.json
for st in 2 3; do
  OVL_PACK_STAGE=$st OVL_TRACE_PIPE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/bench_stage$st.json 2> $OUT/trace_stage$st.txt || { echo "bench failed"; exit 1; }
done
echo done

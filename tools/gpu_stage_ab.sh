#!/bin/bash
# A/B of the packed transport: scoring into HBM + copy kernel (OVL_PACK_STAGE=1) vs stores over the link from
# the scoring kernel (0); pipeline traces of both; the pipeline GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-stage}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_compact_pairs.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in target cfg3; do
  timeout -k 10 300 python -u tools/pack_ab.py $c 5 20 > $OUT/ab_$c.json 2> $OUT/ab_$c.err || { echo "ab $c failed"; tail -20 $OUT/ab_$c.err; exit 1; }
  cat $OUT/ab_$c.json
done
for st in 1 0; do
  OVL_PACK_STAGE=$st OVL_TRACE_PIPE=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/bench_stage$st.json 2> $OUT/trace_stage$st.txt || { echo "bench failed"; exit 1; }
done
echo done

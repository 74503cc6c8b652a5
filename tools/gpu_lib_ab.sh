#!/bin/bash
# A/B of library builds (default build vs build/ablate_<V>/libovl.so): parity subset on the variant first,
# then kernel-only and step time, interleaved passes.   bash tools/gpu_lib_ab.sh TAG VARIANT PASSES [TEST_ON]
# TEST_ON: variant (default) | default (the parity subset runs on the default build instead) | none
# BENCH_ARGS (env): extra bench.py arguments, e.g. "--config cfg3"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$1; V=$2; PASSES=${3:-3}
mkdir -p $OUT
VL="$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd/build/ablate_$V/libovl.so"
TL=$VL; [ "${4:-variant}" = default ] && TL=""
if [ "${4:-variant}" != none ]; then
OVL_LIB_PATH=$TL timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_candidates.py -x -q \
  --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "variant tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
fi
for pass in $(seq 1 $PASSES); do
  for L in default $V; do
    if [ $L = default ]; then LP=""; else LP="OVL_LIB_PATH=$VL"; fi
    env $LP timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-extra $BENCH_ARGS > $OUT/${L}_$pass.json 2>>$OUT/err.log || { echo "bench failed $L"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${L}_$pass.json').read().strip().splitlines()[-1]); print('$L pass $pass kernel_us', round(d['kernel_only_roofline']['kernel_ms']*1000,2), 'step_ms', round(d['ms_per_step'],4), 'in-step packed us', round(d['roofline']['launch_ms']*1000,2))"
  done
done

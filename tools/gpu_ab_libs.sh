# A/B of several libovl builds: parity tests on the first, then kernel event time per config, alternating.
# usage: bash tools/gpu_ab_libs.sh "<lib paths relative to the package dir>" "<configs>" [reps]
set -u
cd "$GRAFT_REPO_ROOT"
LIBS=$1; CFGS=${2:-"cfg2 target cfg3"}; REPS=${3:-2}
P=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/ab/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in $(seq $REPS); do
for lib in $LIBS; do
for cfg in $CFGS; do
  OVL_LIB_PATH=$P/$lib timeout -k 10 300 python bench.py --config $cfg --steps 2000 --warmup 20 --no-extra --no-cpu-baseline > gpurun_out/ab/x.json 2> gpurun_out/ab/x.err || { tail -5 gpurun_out/ab/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'kernel_us %.2f' % (d['roofline']['kernel_ms']*1e3))" gpurun_out/ab/x.json $lib $cfg
done; done; done

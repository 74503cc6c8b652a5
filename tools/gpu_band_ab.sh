# band lane kernel: GPU band tests, then the cfg5 band sweep (kernel time per band) for two builds, alternating
set -u
cd "$GRAFT_REPO_ROOT"
P=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd
mkdir -p gpurun_out/bab
timeout -k 10 900 python -u -m pytest tests/test_gpu_banded.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bab/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/bab/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for lib in build/libovl.so build/ab_old/libovl.so; do
  OVL_LIB_PATH=$P/$lib timeout -k 10 300 python bench.py --config cfg5 --band-sweep 32,40,48,56,64 --sweep-steps 10 --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/bab/x.json 2> gpurun_out/bab/x.err || { tail -5 gpurun_out/bab/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], ' '.join('b%d=%.3f' % (p['band'], p['kernel_ms']) for p in d['band_sweep']['points']))" gpurun_out/bab/x.json $lib
done; done

set -u
cd "$GRAFT_REPO_ROOT"
P=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd
mkdir -p gpurun_out/bab
for rep in 1 2; do
for lib in build/libovl.so build/ab_old/libovl.so; do
  OVL_LIB_PATH=$P/$lib timeout -k 10 300 python bench.py --config cfg5 --band-sweep 64 --sweep-steps 10 --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/bab/x.json 2> gpurun_out/bab/x.err || { tail -5 gpurun_out/bab/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], ' '.join('b%d=%.3f' % (p['band'], p['kernel_ms']) for p in d['band_sweep']['points']))" gpurun_out/bab/x.json $lib
done; done

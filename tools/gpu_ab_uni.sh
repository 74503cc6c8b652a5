# A/B of two libovl builds on the ungapped configs (kernel event time, 2000 steps, alternating).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for rep in 1 2; do
for lib in build/libovl.so build/ab_old/libovl.so; do
for cfg in cfg2 target cfg3; do
  OVL_LIB_PATH=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd/$lib timeout -k 10 300 python bench.py --config $cfg --steps 2000 --warmup 20 --no-extra --no-cpu-baseline > gpurun_out/ab/x.json 2> gpurun_out/ab/x.err || { tail -5 gpurun_out/ab/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'kernel_us %.2f' % (d['roofline']['kernel_ms']*1e3))" gpurun_out/ab/x.json $lib $cfg
done; done; done

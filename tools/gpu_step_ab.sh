# A/B of libovl builds on the metric's step (results in host memory): ms_per_step, alternating builds.
# usage: bash tools/gpu_step_ab.sh "<libs relative to the package dir>" "<configs>" [reps] [steps]
set -u
cd "$GRAFT_REPO_ROOT"
LIBS=$1; CFGS=${2:-"target cfg4"}; REPS=${3:-3}; STEPS=${4:-200}
P=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd
mkdir -p gpurun_out/sab
for rep in $(seq $REPS); do
for lib in $LIBS; do
for cfg in $CFGS; do
  OVL_LIB_PATH=$P/$lib timeout -k 10 300 python bench.py --config $cfg --steps $STEPS --warmup 10 --no-extra --no-cpu-baseline > gpurun_out/sab/x.json 2> gpurun_out/sab/x.err || { tail -5 gpurun_out/sab/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'step_ms %.4f kernel_ms %.4f' % (d['ms_per_step'], d['roofline']['kernel_ms']))" gpurun_out/sab/x.json $lib $cfg
done; done; done

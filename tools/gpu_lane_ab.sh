# A/B of the lane kernel's profile build (v_perm default vs OVL_LANE_MUX build): lane parity on the default
# lib, then the cfg5 full-DP point per lib, alternating.
set -u
cd "$GRAFT_REPO_ROOT"
P=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd
mkdir -p gpurun_out/lane_ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp_lane.py tests/test_gpu_parity.py -k "lane or gapped or dp" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lane_ab/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/lane_ab/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for lib in build/libovl.so build/ab_mux/libovl.so; do
  OVL_LIB_PATH=$P/$lib timeout -k 10 300 python bench.py --config cfg5 --steps 3 --warmup 1 --no-extra --no-cpu-baseline --band-sweep -1 --sweep-steps 5 > gpurun_out/lane_ab/x.json 2> gpurun_out/lane_ab/x.err || { tail -5 gpurun_out/lane_ab/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['band_sweep']['points'][0]; print(sys.argv[2], p['kernel'], round(p['kernel_ms'],3), 'ms', '%.4g cells/s' % p['cells_per_s'])" gpurun_out/lane_ab/x.json $lib
done; done

# Lane-per-pair DP: parity tests, then the cfg5 full-DP point for each kernel variant and the old kernel.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lane
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp_lane.py tests/test_gpu_parity.py -k "lane or gapped or dp" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lane/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/lane/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in "OVL_LANE_CW=32" "OVL_LANE_CW=16" "OVL_LANE_CW=32 OVL_LANE_SFX=0" "OVL_LANE_CW=16 OVL_LANE_SFX=0"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 300 python bench.py --config cfg5 --steps 3 --warmup 1 --no-extra --no-cpu-baseline --band-sweep -1 --sweep-steps 3 > gpurun_out/lane/cfg5_$tag.json 2> gpurun_out/lane/cfg5_$tag.err || { tail -5 gpurun_out/lane/cfg5_$tag.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d['band_sweep']['points'][0]; print(sys.argv[2], round(p['kernel_ms'],2), 'ms', '%.3g cells/s' % p['cells_per_s'])" gpurun_out/lane/cfg5_$tag.json "$v"
done

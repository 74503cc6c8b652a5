# Band knob: parity tests for every form, then the cfg5 sweep with the default forms.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/band
timeout -k 10 600 python -u -m pytest tests/test_gpu_banded.py tests/test_gpu_dp_lane.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/band/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/band/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config cfg5 --steps 3 --warmup 1 --no-extra --no-cpu-baseline --band-sweep 4,8,16,24,32,48,64,-1 --sweep-steps 3 > gpurun_out/band/cfg5_sweep.json 2> gpurun_out/band/cfg5_sweep.err || { tail -5 gpurun_out/band/cfg5_sweep.err; exit 1; }
python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for p in d['band_sweep']['points']: print(p['band'], round(p['kernel_ms'],3), 'ms', '%.3g cells/s' % p['cells_per_s'])
" gpurun_out/band/cfg5_sweep.json

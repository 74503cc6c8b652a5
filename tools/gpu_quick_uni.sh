# Uniform kernel A/B: parity tests of the ungapped path, then cfg2 / target / cfg3 kernel times.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/uni
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/uni/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/uni/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in cfg2 target cfg3; do
  timeout -k 10 300 python bench.py --config $cfg --steps 2000 --warmup 20 --no-extra --no-cpu-baseline > gpurun_out/uni/$cfg.json 2> gpurun_out/uni/$cfg.err || { tail -5 gpurun_out/uni/$cfg.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value %.4g' % d['value'], 'kernel_us %.2f' % (d['roofline']['kernel_ms']*1e3), 'ms_per_step %.4f' % d['ms_per_step'])" gpurun_out/uni/$cfg.json $cfg
done

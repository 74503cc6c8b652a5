# New clustered-side-pair parity test, then latency mode (OVL_SPLIT=1) vs the default at the target point.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/split
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "clustered or split_knob" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/split/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/split/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for sp in default 1; do
for cfg in target cfg3; do
  if [ $sp = default ]; then E=""; else E="OVL_SPLIT=$sp"; fi
  env $E timeout -k 10 300 python bench.py --config $cfg --steps 1000 --warmup 20 --no-extra --no-cpu-baseline > gpurun_out/split/x.json 2> gpurun_out/split/x.err || { tail -5 gpurun_out/split/x.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'kernel_us %.2f' % (d['roofline']['kernel_ms']*1e3))" gpurun_out/split/x.json split=$sp $cfg
done; done; done

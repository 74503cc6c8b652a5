# packed result transport: pipeline + parity GPU tests, host-array entry points A/B (packed / int32 / direct
# share / chunk sizes / store kinds / copy engine) at the target point and cfg2, then the bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pk
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if isinstance(v, dict): print(k, {kk: vv['ms'] for kk, vv in v.items()})
    else: print(k, v)" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_c_abi.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pk/pytest.log 2>&1 || { tail -40 gpurun_out/pk/pytest.log; exit 1; }
tail -2 gpurun_out/pk/pytest.log
timeout -k 10 300 python tools/host_paths_ab.py target 30 > gpurun_out/pk/target.json && show gpurun_out/pk/target.json && \
timeout -k 10 300 python tools/host_paths_ab.py cfg3 20 > gpurun_out/pk/cfg3.json && show gpurun_out/pk/cfg3.json && \
timeout -k 10 300 python bench.py > gpurun_out/pk/bench.log 2>&1 && grep '^{"metric"' gpurun_out/pk/bench.log | python -c "
import json, sys; d = json.loads(sys.stdin.read()); print({k: d[k] for k in ('value', 'ms_per_step')}, d.get('roofline', {}).get('kernel_ms'), {k: v.get('ms_per_step') for k, v in d.get('extra_configs', {}).items() if isinstance(v, dict)})"

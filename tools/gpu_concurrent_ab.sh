# direct chunk concurrent on a second stream (default) vs after the packed chunks (OVL_PACK_CONCURRENT=0):
# pipeline tests, three processes (tools/pack_ab.py), a trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/cc
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print({k: (v['pinned']['median_ms'], v['pageable']['median_ms'], v.get('packed_share_pinned')) for k, v in d.items() if isinstance(v, dict)})" "$1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cc/pytest.log 2>&1 || { tail -30 gpurun_out/cc/pytest.log; exit 1; }
tail -1 gpurun_out/cc/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/cc/a.$i.json && show gpurun_out/cc/a.$i.json || exit 1
done

# two packed chunks sized 1 : g (OVL_PACK_GROWTH), three processes (tools/pack_ab.py), target and cfg3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gr
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print({k: (v['pinned']['median_ms'], v['pageable']['median_ms'], v.get('packed_share_pinned')) for k, v in d.items() if isinstance(v, dict)})" "$1"; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -k packed -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gr/pytest.log 2>&1 || { tail -30 gpurun_out/gr/pytest.log; exit 1; }
tail -1 gpurun_out/gr/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/gr/t.$i.json && show gpurun_out/gr/t.$i.json || exit 1
done
timeout -k 10 300 python tools/pack_ab.py cfg3 4 10 > gpurun_out/gr/c.json && show gpurun_out/gr/c.json

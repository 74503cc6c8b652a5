# adaptive direct share vs fixed 18 % / 25 %: packed tests, then three processes (tools/pack_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ad
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print({k: (v['pinned']['median_ms'], v['pageable']['median_ms'], v.get('packed_share_pinned')) for k, v in d.items() if isinstance(v, dict)})" "$1"; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -k packed -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ad/pytest.log 2>&1 || { tail -30 gpurun_out/ad/pytest.log; exit 1; }
tail -1 gpurun_out/ad/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/ad/a.$i.json && show gpurun_out/ad/a.$i.json || exit 1
done

# host pool placement: unpinned (OVL_POOL_NUMA=0) vs following the destination's NUMA node (default, 2),
# three processes each (tools/pack_ab.py, target point)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/numa
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict)})" "$1" "$2"; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -k "packed or pinned_and_pageable" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/numa/pytest.log 2>&1 || { tail -30 gpurun_out/numa/pytest.log; exit 1; }
tail -1 gpurun_out/numa/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/numa/follow.$i.json && show gpurun_out/numa/follow.$i.json follow || exit 1
  OVL_POOL_NUMA=0 timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/numa/free.$i.json && show gpurun_out/numa/free.$i.json free || exit 1
done

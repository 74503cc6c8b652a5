# packed transport: host pool on the GPU's NUMA node (default) or unpinned (OVL_POOL_NUMA=0), three
# processes each, direct share 0-25 % (tools/pack_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pk
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict)})" "$1" "$2"; }
for i in 1 2 3; do
  timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/pk/ab5_numa_$i.json && show gpurun_out/pk/ab5_numa_$i.json numa || exit 1
  OVL_POOL_NUMA=0 timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/pk/ab5_free_$i.json && show gpurun_out/pk/ab5_free_$i.json free || exit 1
done

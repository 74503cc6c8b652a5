# host pool size: 8 (default) vs 12 vs 6 threads, three processes each, alternating (tools/pack_ab.py);
# prints the job's cgroup CPU limit first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/thr
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict) and k in ('packed_pct18', 'packed_pct25', 'packed_pct0')})" "$1" "$2"; }
for i in 1 2 3; do
  for t in 8 12 6; do
    OVL_HOST_THREADS=$t timeout -k 10 300 python tools/pack_ab.py target 4 20 > gpurun_out/thr/t$t.$i.json && show gpurun_out/thr/t$t.$i.json t$t || exit 1
  done
done

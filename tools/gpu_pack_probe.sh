# packed step: bench.py's Workload timed as bench.py times it vs fresh arrays (tools/bench_step_probe.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pk
timeout -k 10 300 python tools/bench_step_probe.py 50 > gpurun_out/pk/bprobe.json && cat gpurun_out/pk/bprobe.json && \
timeout -k 10 300 python bench.py > gpurun_out/pk/bench.log 2>&1 && grep '^{"metric"' gpurun_out/pk/bench.log | python -c "
import json, sys; d = json.loads(sys.stdin.read()); print({k: d[k] for k in ('value', 'ms_per_step')}, d['host_paths'])"

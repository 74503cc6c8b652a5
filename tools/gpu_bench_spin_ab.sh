# default bench with the host pool polling (default) and sleeping (OVL_POOL_SPIN_US=0), twice each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sp
show() { grep '^{"metric"' "$1" | python -c "
import json, sys; d = json.loads(sys.stdin.read())
print(sys.argv[1], round(d['ms_per_step'], 4), {k: round(v['ms_per_step'], 4) for k, v in d['extra_configs'].items() if isinstance(v, dict) and 'ms_per_step' in v}, {k: round(v['ms_per_call'], 4) for k, v in d['host_paths'].items() if isinstance(v, dict)})" "$2"; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/sp/spin_$i.log 2>&1 && show gpurun_out/sp/spin_$i.log spin || exit 1
  OVL_POOL_SPIN_US=0 timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/sp/sleep_$i.log 2>&1 && show gpurun_out/sp/sleep_$i.log sleep || exit 1
done

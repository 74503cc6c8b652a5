# direct share of the packed step with the default pool (12 threads): three processes (tools/pack_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pct
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print({k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict)})" "$1"; }
for i in 1 2 3; do
  timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/pct/pct.$i.json && show gpurun_out/pct/pct.$i.json || exit 1
done

# packed transport below the 1 M-pair threshold (PACK_AB_MIN0=1): cfg2 (122 K pairs), twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/small
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print({k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict)})" "$1"; }
for i in 1 2; do
  PACK_AB_MIN0=1 timeout -k 10 300 python tools/pack_ab.py cfg2 5 100 > gpurun_out/small/cfg2.$i.json && show gpurun_out/small/cfg2.$i.json || exit 1
done

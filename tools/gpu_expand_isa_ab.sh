# packed step with the host expansion at each vector width (OVL_EXPAND_ISA, read once per process), two
# processes each, interleaved settings inside each (tools/pack_ab.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/isa
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print(sys.argv[2], {k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict)})" "$1" "$2"; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -k packed -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/isa/pytest.log 2>&1 || { tail -30 gpurun_out/isa/pytest.log; exit 1; }
tail -1 gpurun_out/isa/pytest.log
for i in 1 2; do
  for isa in sse2 avx2 avx512; do
    OVL_EXPAND_ISA=$isa timeout -k 10 300 python tools/pack_ab.py target 5 20 > gpurun_out/isa/$isa.$i.json && show gpurun_out/isa/$isa.$i.json $isa || exit 1
  done
done

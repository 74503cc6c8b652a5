# polled packed expansion: pipeline / parity / C ABI GPU tests, interleaved A/B and the pipeline trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pp
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
print({k: (v['pinned']['median_ms'], v['pageable']['median_ms']) for k, v in d.items() if isinstance(v, dict)})" "$1"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_c_abi.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pp/pytest.log 2>&1 || { tail -40 gpurun_out/pp/pytest.log; exit 1; }
tail -2 gpurun_out/pp/pytest.log
timeout -k 10 300 python tools/pack_ab.py target 7 20 > gpurun_out/pp/ab_1.json && show gpurun_out/pp/ab_1.json && \
timeout -k 10 300 python tools/pack_ab.py target 7 20 > gpurun_out/pp/ab_2.json && show gpurun_out/pp/ab_2.json && \
timeout -k 10 300 python tools/pack_ab.py cfg3 5 10 > gpurun_out/pp/ab_cfg3.json && show gpurun_out/pp/ab_cfg3.json && \
OVL_TRACE_PIPE=1 timeout -k 10 300 python tools/pack_ab.py target 2 10 > /dev/null 2> gpurun_out/pp/trace.txt && \
python - <<'PY'
import collections, re
lines = [l for l in open("gpurun_out/pp/trace.txt") if l.startswith("ovl_pipe:")]
groups = collections.defaultdict(list)
for l in lines:
    ev = re.findall(r"(\w\d+)=([\d.]+)", l)
    groups[" ".join(k for k, _ in ev)].append([float(v) for _, v in ev])
for key, rows in groups.items():
    med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
    print(len(rows), " ".join(f"{k}={v:.0f}" for k, v in zip(key.split(), med)))
PY

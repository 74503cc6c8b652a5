# pipeline event trace (OVL_TRACE_PIPE=1) of the target-point step into pinned arrays, after warm-up
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/tr
OVL_TRACE_PIPE=1 timeout -k 10 300 python tools/pack_ab.py target 2 10 > gpurun_out/tr/ab.json 2> gpurun_out/tr/trace.txt && \
python - <<'PY'
import collections, re
lines = [l for l in open("gpurun_out/tr/trace.txt") if l.startswith("ovl_pipe:")]
groups = collections.defaultdict(list)
for l in lines:
    ev = re.findall(r"(\w\d+)=([\d.]+)", l)
    groups[" ".join(k for k, _ in ev)].append([float(v) for _, v in ev])
for key, rows in groups.items():
    med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
    print(len(rows), " ".join(f"{k}={v:.0f}" for k, v in zip(key.split(), med)))
PY

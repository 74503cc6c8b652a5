# packed transport settings interleaved in one process (tools/pack_ab.py) at the target point, with the
# host pool at 8 (default), 12 and 16 threads (OVL_HOST_THREADS is read once per process)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pk
show() { python -c "
import json, sys; d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if isinstance(v, dict): print(k, {kk: vv['median_ms'] for kk, vv in v.items()})
    else: print(k, v)" "$1"; }
timeout -k 10 400 python tools/pack_ab.py target 7 20 > gpurun_out/pk/ab2_t8.json && show gpurun_out/pk/ab2_t8.json && \
OVL_HOST_THREADS=12 timeout -k 10 400 python tools/pack_ab.py target 7 20 > gpurun_out/pk/ab2_t12.json && show gpurun_out/pk/ab2_t12.json && \
OVL_HOST_THREADS=16 timeout -k 10 400 python tools/pack_ab.py target 7 20 > gpurun_out/pk/ab2_t16.json && show gpurun_out/pk/ab2_t16.json && \
OVL_HOST_THREADS=4 timeout -k 10 400 python tools/pack_ab.py target 7 20 > gpurun_out/pk/ab2_t4.json && show gpurun_out/pk/ab2_t4.json

"""A/B of the host-result path at the target point (tools/gpu_pipe_ab.sh): kernel stores straight into
pinned host memory (OVL_PIPE_DIRECT=1, coherent / non-coherent / default host memory) vs chunked D2H
copies (OVL_PIPE_DIRECT=0, several chunk sizes), plus a raw 16 MB D2H copy for the link rate."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ovlgraph import OverlapEngine  # noqa: E402
from ovlgraph.candidates import dedup_reads  # noqa: E402
from ovlgraph.hostmem import PinnedPool  # noqa: E402
from ovlgraph.reads import config_reads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
reads, _ = dedup_reads(config_reads(cfg, seed=0))
torch.cuda.set_device(0)
res = {"config": cfg}

# raw link rate: one 16 MB device->pinned copy
x = torch.ones(4 << 20, dtype=torch.int32, device="cuda")
h = torch.empty(4 << 20, dtype=torch.int32, pin_memory=True)
for _ in range(3):
    h.copy_(x, non_blocking=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    h.copy_(x, non_blocking=True)
torch.cuda.synchronize()
res["raw_d2h_16MB_GBs"] = 20 * x.numel() * 4 / (time.perf_counter() - t0) / 1e9

settings = [("direct_default", {"OVL_PIPE_DIRECT": "1"}),
            ("direct_coherent", {"OVL_PIPE_DIRECT": "1", "OVL_HOST_COHERENT": "1"}),
            ("direct_noncoherent", {"OVL_PIPE_DIRECT": "1", "OVL_HOST_COHERENT": "0"}),
            ("copy_auto", {"OVL_PIPE_DIRECT": "0"}),
            ("copy_125k", {"OVL_PIPE_DIRECT": "0", "OVL_PIPE_CHUNK": "131072"}),
            ("copy_500k", {"OVL_PIPE_DIRECT": "0", "OVL_PIPE_CHUNK": "524288"}),
            ("copy_1chunk", {"OVL_PIPE_DIRECT": "0", "OVL_PIPE_CHUNK": "4194304"})]
ref = None
for name, env in settings:
    keep = {k: os.environ.get(k) for k in ("OVL_PIPE_DIRECT", "OVL_HOST_COHERENT", "OVL_PIPE_CHUNK")}
    for k in keep:
        os.environ.pop(k, None)
    os.environ.update(env)
    eng = OverlapEngine(0)
    pool = PinnedPool()
    eng.set_reads(reads)
    n = eng.enumerate_candidates(5)
    out = (pool.empty(n), pool.empty(n))
    for _ in range(3):
        eng.score_candidates(out=out)
    t0 = time.perf_counter()
    reps = 30
    for _ in range(reps):
        eng.score_candidates(out=out)
    dt = (time.perf_counter() - t0) / reps
    eng.set_timing(True)
    eng.score_candidates(out=out)
    km = eng.last_timing()["kernel_ms"]
    eng.set_timing(False)
    if ref is None:
        ref = (out[0].copy(), out[1].copy())
    same = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
    res[name] = {"ms": dt * 1e3, "pairs_per_s": n / dt, "kernel_ms_in_call": km, "same": same,
                 "result_GBs": 8 * n / dt / 1e9}
    eng.close()
    del out
    pool.trim()
    for k, v in keep.items():
        os.environ.pop(k, None)
        if v is not None:
            os.environ[k] = v
print(json.dumps(res, indent=1))

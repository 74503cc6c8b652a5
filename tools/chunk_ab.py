"""The step (resident list -> pinned host results, direct stores) with the list cut into chunks launched
back to back on one stream (OVL_PIPE_CHUNK): does a later chunk's sweep overlap an earlier chunk's result
stores draining over PCIe, hiding the first tile's latency?

    python tools/chunk_ab.py [config] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import CONFIGS, config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    res, ref = {"config": cfg}, None
    for chunk in (0, 65536, 131072, 262144, 524288, 1048576, 0):
        if chunk:
            os.environ["OVL_PIPE_CHUNK"] = str(chunk)
        else:
            os.environ.pop("OVL_PIPE_CHUNK", None)
        eng = OverlapEngine(0)
        os.environ.pop("OVL_PIPE_CHUNK", None)
        eng.set_reads(reads)
        n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
        out = (pinned_empty(n), pinned_empty(n))
        for _ in range(5):
            eng.score_candidates(out=out)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.score_candidates(out=out)
        dt = (time.perf_counter() - t0) / reps
        if ref is None:
            ref = (out[0].copy(), out[1].copy())
        same = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
        res.setdefault(str(chunk or "whole"), []).append({"ms": round(dt * 1e3, 4), "same": same})
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

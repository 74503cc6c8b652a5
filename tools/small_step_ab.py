"""Small lists (cfg2): the step (results into pinned host memory) under different launch shapes, set through
the tuning knobs read at context creation: OVL_SPLIT (0 = one wavefront per tile, 1 = latency mode) and
OVL_BLOCKS_PER_CU (grid cap).  Fewer concurrent wavefronts finish their first tiles sooner, so results can
start crossing PCIe before the whole list is swept.

    python tools/small_step_ab.py [config] [reps]
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    settings = [("auto", {}), ("lat", {"OVL_SPLIT": "1"}), ("thr_bpc32", {"OVL_SPLIT": "0"}),
                ("thr_bpc8", {"OVL_SPLIT": "0", "OVL_BLOCKS_PER_CU": "8"}),
                ("thr_bpc4", {"OVL_SPLIT": "0", "OVL_BLOCKS_PER_CU": "4"}),
                ("thr_bpc2", {"OVL_SPLIT": "0", "OVL_BLOCKS_PER_CU": "2"}),
                ("thr_bpc1", {"OVL_SPLIT": "0", "OVL_BLOCKS_PER_CU": "1"}),
                ("lat_bpc2", {"OVL_SPLIT": "1", "OVL_BLOCKS_PER_CU": "2"}),
                ("auto", {})]
    res, ref = {"config": cfg}, None
    for name, env in settings:
        for k in ("OVL_SPLIT", "OVL_BLOCKS_PER_CU"):
            os.environ.pop(k, None)
        os.environ.update(env)
        eng = OverlapEngine(0)
        for k in ("OVL_SPLIT", "OVL_BLOCKS_PER_CU"):
            os.environ.pop(k, None)
        eng.set_reads(reads)
        n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
        out = (pinned_empty(n), pinned_empty(n))
        for _ in range(20):
            eng.score_candidates(out=out)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.score_candidates(out=out)
        dt = (time.perf_counter() - t0) / reps
        eng.set_timing(True)
        ks = []
        for _ in range(50):
            eng.score_candidates(out=out)
            ks.append(eng.last_timing()["kernel_ms"])
        eng.set_timing(False)
        if ref is None:
            ref = (out[0].copy(), out[1].copy())
        same = bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1]))
        res.setdefault(name, []).append({"step_us": round(dt * 1e6, 2), "kernel_in_call_us": round(float(np.median(ks)) * 1e3, 2),
                                         "same": same})
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

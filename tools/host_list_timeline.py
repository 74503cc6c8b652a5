"""GPU timeline of host-pair-list calls (for rocprofv3 --kernel-trace): ovl_score_host with the target list in
pinned host memory (compact encoding), `reps` calls after 3 warm-up calls, with a 2 ms gap between calls so
that each call's kernels group apart in the trace.

    rocprofv3 --kernel-trace -d DIR -o tl -- python3 tools/host_list_timeline.py [config] [reps]
"""
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
    from ovlgraph.reads import config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    eng = OverlapEngine(0)
    eng.set_reads(reads)
    a, b = eng.candidates(5)
    a, b = np.array(a), np.array(b)
    pa, pb = pinned_empty(a.shape[0]), pinned_empty(a.shape[0])
    pa[:], pb[:] = a, b
    out = (pinned_empty(a.shape[0]), pinned_empty(a.shape[0]))
    for _ in range(3):
        eng.score(pa, pb, out=out)
    ts = []
    for _ in range(reps):
        time.sleep(0.002)
        t0 = time.perf_counter()
        eng.score(pa, pb, out=out)
        ts.append((time.perf_counter() - t0) * 1e3)
    print({"ms": [round(t, 4) for t in ts], "median_ms": float(np.median(ts))})
    eng.close()


if __name__ == "__main__":
    main()

"""Resident grid latency on the box (diagnostic): rank 0's shard of the target list at N = 1 and 8 scored through the
resident grid under each record store form (ovl_grid.h kResidentStore*) and blocks per CU, back to back; with
OVL_TRACE_PIPE=1 every call's stderr line gives when its first record, half, 90 %, 99 % and all of its tiles were
taken (microseconds after the post).

    OVL_TRACE_PIPE=1 python tools/resident_probe.py "1x2x4,1x4x4,..." [calls]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))


def main():
    import numpy as np
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import config_reads
    forms = sys.argv[1].split(",")
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    reads, _ = dedup_reads(config_reads("target", seed=0))
    res = []
    for form in forms:
        os.environ["OVL_RESIDENT"] = form
        eng = OverlapEngine(0)
        os.environ.pop("OVL_RESIDENT")
        eng.set_reads(reads)
        n = eng.enumerate_candidates(5)
        out = (pinned_empty(n), pinned_empty(n))
        ref = eng.score_candidates()
        ref = (np.array(ref[0]), np.array(ref[1]))
        for N in (8, 1):
            lo, hi = eng.candidate_shards(N)[:2]
            o = (out[0][lo:hi], out[1][lo:hi])
            step = eng.range_scorer(lo, hi, o)
            print(f"== {form} N={N}", file=sys.stderr, flush=True)
            for _ in range(10):
                step()
            ts = []
            for _ in range(calls):
                t0 = time.perf_counter()
                step()
                ts.append(time.perf_counter() - t0)
            ok = bool(np.array_equal(o[0], ref[0][lo:hi]) and np.array_equal(o[1], ref[1][lo:hi]))
            res.append({"form": form, "ranks": N, "pairs": hi - lo, "median_ms": round(float(np.median(ts)) * 1e3, 4),
                        "min_ms": round(float(np.min(ts)) * 1e3, 4), "exact": ok, "stats": eng.resident_stats()})
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

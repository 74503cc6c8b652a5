"""Packed vs int32 results by list size: ovl_score_candidates_range over the first n pairs of the target
point's resident list into pinned arrays, both engines interleaved (OVL_PACK_MIN=0 vs OVL_PACK=0).

    python tools/pack_size_ab.py [rounds] [reps]
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
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    reads, _ = dedup_reads(config_reads("target", seed=0))
    engines = {}
    for name, env in (("int32", {"OVL_PACK": "0"}), ("packed", {"OVL_PACK_MIN": "0"})):
        os.environ.update(env)
        eng = OverlapEngine(0)
        for k in env:
            os.environ.pop(k, None)
        eng.set_reads(reads)
        eng.enumerate_candidates(CONFIGS["target"]["k"])
        engines[name] = eng
    sizes = [131072, 262144, 524288, 786432, 1048576]
    out = (pinned_empty(sizes[-1]), pinned_empty(sizes[-1]))
    t = {(s, e): [] for s in sizes for e in engines}
    for _ in range(rounds):
        for s in sizes:
            o = (out[0][:s], out[1][:s])
            for name, eng in engines.items():
                for _ in range(3):
                    eng.score_candidates_range(0, s, out=o)
                t0 = time.perf_counter()
                for _ in range(reps):
                    eng.score_candidates_range(0, s, out=o)
                t[(s, name)].append((time.perf_counter() - t0) / reps * 1e3)
    res = {str(s): {e: round(float(np.median(t[(s, e)])), 4) for e in engines} for s in sizes}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

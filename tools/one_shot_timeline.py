"""The §8(d)-literal one-shot call (ovl_score_pairs: reads uploaded and packed, host pair list, results into
pinned arrays) at the target point, with OVL_TRACE_PIPE=1 set by the caller: stderr gets one line of
microsecond marks per set_reads (r recount, p prepared, s staged, u uploads issued, y synchronised) and per
scoring pipeline (s setup, e<k> chunk k encoded, i<k> issued, w<k> results ready, d<k> drained, y synchronised).
Prints the median wall time of each call kind.

    OVL_TRACE_PIPE=1 python tools/one_shot_timeline.py [reps]
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
    from ovlgraph.engine import encode_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import config_reads
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    reads, _ = dedup_reads(config_reads("target", seed=0))
    enc = encode_reads(reads)
    eng = OverlapEngine(0)
    eng.set_reads(reads, enc)
    n = eng.enumerate_candidates(5)
    a, b = eng.candidates_copy(n)
    out = (pinned_empty(n), pinned_empty(n))
    t = {"set_reads": [], "score_host": [], "score_pairs": []}
    for _ in range(reps):
        for kind in t:
            time.sleep(0.002)
            sys.stderr.write(f"== {kind}\n")
            sys.stderr.flush()
            t0 = time.perf_counter()
            if kind == "set_reads":
                eng.set_reads(reads, enc)
            elif kind == "score_host":
                eng.score(a, b, out=out)
            else:
                eng.score_pairs(reads, a, b, out=out, encoded=enc)
            t[kind].append((time.perf_counter() - t0) * 1e3)
    print({k: round(float(np.median(v)), 4) for k, v in t.items()})
    eng.close()


if __name__ == "__main__":
    main()

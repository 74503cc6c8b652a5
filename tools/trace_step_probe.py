"""One traced scoring call after another (OVL_TRACE_PIPE=1 prints each call's pipeline events on stderr): the whole
target list into pinned arrays, or rank r's shard of N (python tools/trace_step_probe.py [N [r]]).  Prints the
median step time and the last call's transfer on stderr."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "genome-assembly-using-overlap-graphs_amd"))


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import config_reads
    shards = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    r = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    reads, _ = dedup_reads(config_reads("target", seed=0))
    eng = OverlapEngine(0)
    eng.set_reads(reads)
    n = eng.enumerate_candidates(5)
    cuts = eng.candidate_shards(shards)
    lo, hi = int(cuts[r]), int(cuts[r + 1])
    out = (pinned_empty(n), pinned_empty(n))
    o = (out[0][lo:hi], out[1][lo:hi])
    for _ in range(60):
        eng.score_candidates_range(lo, hi, out=o)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        eng.score_candidates_range(lo, hi, out=o)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print("pairs", hi - lo, "median ms", ts[len(ts) // 2] * 1e3, "transfer", eng.last_transfer(), file=sys.stderr)
    eng.close()


if __name__ == "__main__":
    main()

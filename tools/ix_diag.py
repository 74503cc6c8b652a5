"""Which path a host pair list takes (ovl_last_pair_list), chunk plan and link bytes, at the target point."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.engine import host_pool
    from ovlgraph.reads import config_reads
    print({k: v for k, v in os.environ.items() if k.startswith("OVL")}, host_pool())
    reads, _ = dedup_reads(config_reads("target", seed=0))
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        n = eng.enumerate_candidates(5)
        a, b = eng.candidates_copy(n)
        import numpy as np
        a, b = np.array(a), np.array(b)
        eng.set_timing(True)
        for m in (n, 400_000, 150_000):
            eng.score(a[:m], b[:m])
            print(m, eng.last_pair_list(), eng.last_transfer(), eng.info(),
                  [(r["sink"], r["pairs"]) for r in eng.last_launches()], flush=True)


if __name__ == "__main__":
    main()

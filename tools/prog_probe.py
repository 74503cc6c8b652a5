"""Progressive transport probe: kernel time inside the call (ovl_set_timing) and call time, progressive vs the
chunked packed pipeline, target point, pinned arrays; OVL_PG_* knobs are read per context.

    python tools/prog_probe.py [config]
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
    from ovlgraph.reads import config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    res = {}
    for name, env in (("chunked", {"OVL_PROGRESSIVE": "0"}),
                      ("prog_dev", {"OVL_PROGRESSIVE": "1", "OVL_PG_STORE": "1"}),
                      ("prog_dev_nowait", {"OVL_PROGRESSIVE": "1", "OVL_PG_STORE": "5"}),
                      ("prog_sys_nowait", {"OVL_PROGRESSIVE": "1", "OVL_PG_STORE": "4"}),
                      ("prog_nt_nowait", {"OVL_PROGRESSIVE": "1", "OVL_PG_STORE": "6"}),
                      ("chunked2", {"OVL_PROGRESSIVE": "0"})):
        os.environ.update(env)
        eng = OverlapEngine(0)
        eng.set_reads(reads)
        n = eng.enumerate_candidates(5)
        out = (pinned_empty(n), pinned_empty(n))
        for _ in range(5):
            eng.score_candidates(out=out)
        eng.set_timing(True)
        ks, cs = [], []
        for _ in range(20):
            t0 = time.perf_counter()
            eng.score_candidates(out=out)
            cs.append((time.perf_counter() - t0) * 1e3)
            ks.append(eng.last_timing()["kernel_ms"])
        eng.set_timing(False)
        t0 = time.perf_counter()
        for _ in range(20):
            eng.score_candidates(out=out)
        res[name] = {"kernel_ms_median": float(np.median(ks)), "call_ms_timed_median": float(np.median(cs)),
                     "call_ms_untimed": (time.perf_counter() - t0) / 20 * 1e3}
        eng.close()
        for k in env:
            os.environ.pop(k, None)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Packed-result step (resident list -> host arrays) as the bench runs it: torch initialises the GPU first,
then engines with polled or blocking pipeline waits (OVL_SPIN_WAIT) and packed or int32 results (OVL_PACK).

    python tools/pack_torch_probe.py [config] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def main():
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import CONFIGS, config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    res = {"config": cfg}
    ref = None
    for name, env in (("spin_packed", {}), ("block_packed", {"OVL_SPIN_WAIT": "0"}),
                      ("spin_int32", {"OVL_PACK": "0"}), ("block_int32", {"OVL_PACK": "0", "OVL_SPIN_WAIT": "0"}),
                      ("spin_packed_again", {})):
        for k in ("OVL_SPIN_WAIT", "OVL_PACK"):
            os.environ.pop(k, None)
        os.environ.update(env)
        eng = OverlapEngine(0)
        for k in ("OVL_SPIN_WAIT", "OVL_PACK"):
            os.environ.pop(k, None)
        eng.set_reads(reads)
        n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
        out = (pinned_empty(n), pinned_empty(n))
        pg = (np.empty(n, np.int32), np.empty(n, np.int32))
        r = {}
        for oname, o in (("pinned", out), ("pageable", pg)):
            for _ in range(5):
                eng.score_candidates(out=o)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                eng.score_candidates(out=o)
            torch.cuda.synchronize()
            r[oname] = round((time.perf_counter() - t0) / reps * 1e3, 4)
            if ref is None:
                ref = (o[0].copy(), o[1].copy())
            r[oname + "_same"] = bool(np.array_equal(o[0], ref[0]) and np.array_equal(o[1], ref[1]))
        res[name] = r
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

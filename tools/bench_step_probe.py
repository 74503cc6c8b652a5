"""bench.py's Workload step timed as bench.py times it, against the same call on fresh pinned / pageable
arrays (narrows a bench-vs-probe difference in the packed step).

    python tools/bench_step_probe.py [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def main():
    import torch
    import bench
    from ovlgraph.hostmem import pinned_empty
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    w = bench.Workload("target", seed=0, dev=dev)
    res = {}
    res["bench_timed_steps_ms"] = bench.timed_steps(w.step, reps, 5, dev, 1) / reps * 1e3
    n = w.n_pairs

    def t(o):
        for _ in range(5):
            w.eng.score_candidates(10, -1, w.indel, w.band, out=o)
        t0 = time.perf_counter()
        for _ in range(reps):
            w.eng.score_candidates(10, -1, w.indel, w.band, out=o)
        return (time.perf_counter() - t0) / reps * 1e3

    fresh = (pinned_empty(n), pinned_empty(n))
    pg = (np.empty(n, np.int32), np.empty(n, np.int32))
    for k in range(3):  # alternations: run-to-run noise within one process
        res[f"same_out_ms_{k}"] = t(w.out)
        res[f"fresh_pinned_ms_{k}"] = t(fresh)
        res[f"pageable_ms_{k}"] = t(pg)
    res["out_ptrs"] = [hex(w.out[0].ctypes.data), hex(w.out[1].ctypes.data)]
    res["bench_timed_steps_again_ms"] = bench.timed_steps(w.step, reps, 5, dev, 1) / reps * 1e3
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()

"""Heavy tiles first (uniform_kernel over the resident candidate list) vs list order (OVL_HEAVY_FIRST=0):
the dominant kernel alone (device outputs, HIP events on its stream) over the target point's list, both
engines interleaved, and the step into pinned arrays.

    python tools/heavy_first_ab.py [config] [rounds] [reps]
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
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import CONFIGS, config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    engines = {}
    for name, env in (("heavy_first", {}), ("list_order", {"OVL_HEAVY_FIRST": "0"})):
        os.environ.update(env)
        eng = OverlapEngine(0)
        for k in env:
            os.environ.pop(k, None)
        eng.set_reads(reads)
        n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
        engines[name] = eng
    ds = torch.empty(n, dtype=torch.int32, device=dev)
    de = torch.empty(n, dtype=torch.int32, device=dev)
    out = (pinned_empty(n), pinned_empty(n))
    kt = {k: [] for k in engines}
    st = {k: [] for k in engines}
    res_same = True
    ref = None
    for _ in range(rounds):
        for name, eng in engines.items():
            pa, pb, _ = eng.candidates_device()
            launch = lambda: eng.score_device(pa, pb, n, ds.data_ptr(), de.data_ptr(),  # noqa: E731
                                              stream=stream.cuda_stream)
            for _ in range(3):
                launch()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                launch()
            e1.record(stream)
            torch.cuda.synchronize()
            kt[name].append(e0.elapsed_time(e1) / reps * 1e3)
            got = (ds.cpu().numpy(), de.cpu().numpy())
            if ref is None:
                ref = got
            res_same = res_same and np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
            for _ in range(3):
                eng.score_candidates(out=out)
            t0 = time.perf_counter()
            for _ in range(reps):
                eng.score_candidates(out=out)
            st[name].append((time.perf_counter() - t0) / reps * 1e3)
            res_same = res_same and np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1])
    res = {"config": cfg, "pairs": int(n), "same": bool(res_same)}
    for name in engines:
        res[name] = {"kernel_us_median": round(float(np.median(kt[name])), 2),
                     "kernel_us": [round(x, 2) for x in kt[name]],
                     "step_ms_median": round(float(np.median(st[name])), 4)}
    for eng in engines.values():
        eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

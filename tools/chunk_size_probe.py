"""The uniform kernel alone (HBM output, ovl_score_device) over parts of the target list of the sizes the step's
chunks have: is the in-step chunk's lower rate (DESIGN §4.1, 43 against 32 us per M pairs) the chunk's size -- a
launch's ramp and tail over fewer tiles -- or something the step does beside it?

    python tools/chunk_size_probe.py [rounds] [reps]  -> JSON on stdout

Each size is timed by HIP events on the launch stream, rounds interleaved; the part starts at pair 0 (the heavy
tiles -- the ones holding side pairs -- are scheduled first in every launch over the resident list) and, for the
chunk sizes, also at the list's middle (the step's second packed chunk).
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "genome-assembly-using-overlap-graphs_amd"))


def main():
    import torch
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import config_reads
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    reads, _ = dedup_reads(config_reads("target", seed=0))
    eng = OverlapEngine(0)
    eng.set_reads(reads)
    n = eng.enumerate_candidates(5)
    pa, pb, _ = eng.candidates_device()
    dev = torch.device("cuda", 0)
    ds = torch.empty(n, dtype=torch.int32, device=dev)
    de = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    half = (n // 2) & ~63
    parts = [("whole", 0, n)]
    for m in (1 << 18, 1 << 19, 940_000, 1 << 20, 1_500_000):
        m = (m // 64) * 64
        parts.append((f"first_{m}", 0, m))
        if m <= n - half:
            parts.append((f"middle_{m}", half, half + m))
    times = {p[0]: [] for p in parts}
    for _ in range(rounds):
        for name, lo, hi in parts:
            args = (pa + 4 * lo, pb + 4 * lo, hi - lo, ds.data_ptr() + 4 * lo, de.data_ptr() + 4 * lo)
            for _ in range(3):
                eng.score_device(*args, stream=stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                eng.score_device(*args, stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            times[name].append(e0.elapsed_time(e1) / reps * 1e3)
    eng.check_device_errors()
    out = {"workload": "target point, uniform_kernel alone (ovl_score_device, HBM output)", "pairs": n,
           "rounds": rounds, "reps": reps, "parts": []}
    for name, lo, hi in parts:
        us = float(np.median(times[name]))
        out["parts"].append({"part": name, "lo": lo, "pairs": hi - lo, "median_us": round(us, 2),
                             "min_us": round(min(times[name]), 2),
                             "us_per_M_pairs": round(us / ((hi - lo) / 1e6), 2)})
    eng.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

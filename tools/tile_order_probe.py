"""Does the order of side pairs (read a shorter than the dominant length: scored through the wavefronts'
LDS rings) change the uniform kernel's time?  The target point's list scored kernel-only (device outputs,
HIP events on the launch stream) in its reference order, with the side pairs moved first, moved last, and
with the tiles shuffled; results un-permuted and compared with the reference-order run.

    python tools/tile_order_probe.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def main():
    import torch
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import CONFIGS, config_reads
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    reads, _ = dedup_reads(config_reads("target", seed=0))
    eng = OverlapEngine(0)
    eng.set_reads(reads)
    eng.enumerate_candidates(CONFIGS["target"]["k"])
    a, b = (np.array(x) for x in eng.candidates(CONFIGS["target"]["k"]))
    n = a.shape[0]
    lens = np.array([len(r) for r in reads])
    side = lens[a] < lens.max()
    idx = np.arange(n)
    rng = np.random.default_rng(0)
    tiles = rng.permutation((n + 63) // 64)
    shuffled = np.concatenate([idx[t * 64:(t + 1) * 64] for t in tiles])
    orders = {"reference": idx,
              "side_first": np.concatenate([idx[side], idx[~side]]),
              "side_last": np.concatenate([idx[~side], idx[side]]),
              "tiles_shuffled": shuffled}
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    ref = None
    res = {"pairs": int(n), "side_pairs": int(side.sum())}
    for name, order in orders.items():
        ta = torch.from_numpy(a[order].astype(np.int32)).to(dev)
        tb = torch.from_numpy(b[order].astype(np.int32)).to(dev)
        ds = torch.empty(n, dtype=torch.int32, device=dev)
        de = torch.empty(n, dtype=torch.int32, device=dev)
        launch = lambda: eng.score_device(ta.data_ptr(), tb.data_ptr(), n, ds.data_ptr(), de.data_ptr(),  # noqa: E731
                                          stream=stream.cuda_stream)
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                launch()
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / reps * 1e3)
        sc = np.empty(n, np.int32)
        en = np.empty(n, np.int32)
        sc[order] = ds.cpu().numpy()
        en[order] = de.cpu().numpy()
        if ref is None:
            ref = (sc, en)
        res[name] = {"kernel_us": [round(t, 2) for t in times],
                     "same": bool(np.array_equal(sc, ref[0]) and np.array_equal(en, ref[1]))}
    eng.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

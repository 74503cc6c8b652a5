"""Kernel time against call size at the target point: for each n, the first n pairs of the resident
candidate list scored (a) into HBM (score_device: the kernel alone, OM 0) and (b) into pinned host arrays (the
step's path: packed chunks + direct chunk, score_candidates_range(0, n)).  Run under
``rocprofv3 --kernel-trace --stats`` to read each launch's duration by grid size; the script itself prints the
wall time per call of both.

    python tools/size_probe.py [reps]          SIZE_PROBE_NS="65536,131072,..."   SIZE_PROBE_CONFIG=target
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cfg = os.environ.get("SIZE_PROBE_CONFIG", "target")
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    eng = OverlapEngine(0)
    eng.set_reads(reads)
    n_all = eng.enumerate_candidates(CONFIGS[cfg]["k"])
    ns = [int(x) for x in os.environ.get(
        "SIZE_PROBE_NS", "65536,131072,172032,249856,499712,786432,917504,1048576,%d" % n_all).split(",")]
    pa, pb, _ = eng.candidates_device()
    dev = torch.device("cuda", 0)
    ds = torch.empty(n_all, dtype=torch.int32, device=dev)
    de = torch.empty(n_all, dtype=torch.int32, device=dev)
    out = (pinned_empty(n_all), pinned_empty(n_all))
    ref = eng.score_candidates()
    ref = (np.array(ref[0]), np.array(ref[1]))
    st = torch.cuda.Stream(dev)
    res = []
    for n in ns:
        n = min(n, n_all)
        for _ in range(5):
            eng.score_device(pa, pb, n, ds.data_ptr(), de.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.score_device(pa, pb, n, ds.data_ptr(), de.data_ptr(), stream=st.cuda_stream)
        st.synchronize()
        t_dev = (time.perf_counter() - t0) / reps * 1e3
        o = (out[0][:n], out[1][:n])
        for _ in range(20):
            eng.score_candidates_range(0, n, out=o)
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.score_candidates_range(0, n, out=o)
        t_host = (time.perf_counter() - t0) / reps * 1e3
        assert np.array_equal(o[0], ref[0][:n]) and np.array_equal(o[1], ref[1][:n]), n
        assert np.array_equal(ds[:n].cpu().numpy(), ref[0][:n]) and np.array_equal(de[:n].cpu().numpy(), ref[1][:n])
        eng.set_timing(True)
        eng.score_candidates_range(0, n, out=o)
        plan = [(r["sink"], r["pairs"], round(r["ms"], 4)) for r in eng.last_launches()]
        eng.set_timing(False)
        res.append({"pairs": n, "device_out_ms_per_call": round(t_dev, 4), "host_out_ms_per_call": round(t_host, 4),
                    "host_launches_sink_pairs_ms": plan})
        print(json.dumps(res[-1]), file=sys.stderr, flush=True)
    eng.close()
    print(json.dumps({"config": cfg, "reps": reps, "results": res}))


if __name__ == "__main__":
    main()

"""Kernel time over a config's whole candidate list, device outputs (ovl_score_device, HIP events on the launch
stream): the ungapped plan and, with BANDS, the band knob's launches (its seed and band kernels).  For A/B builds
(OVL_LIB_PATH names the library).   python tools/kernel_alone_probe.py [config] [reps]   -> JSON on stdout"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "genome-assembly-using-overlap-graphs_amd"))


def main():
    import torch
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import CONFIGS, config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    bands = [int(b) for b in os.environ.get("BANDS", "").split(",") if b]
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    eng = OverlapEngine(0)
    eng.set_reads(reads)
    n = eng.enumerate_candidates(CONFIGS[cfg]["k"])
    pa, pb, _ = eng.candidates_device()
    dev = torch.device("cuda", 0)
    ds = torch.empty(n, dtype=torch.int32, device=dev)
    de = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    out = {"config": cfg, "pairs": n, "lib": os.environ.get("OVL_LIB_PATH", "default"), "ms": {}}
    for band in [None] + bands:
        args = (10, -1, -2, band) if band is not None else (10, -1)
        for _ in range(2):
            eng.score_device(pa, pb, n, ds.data_ptr(), de.data_ptr(), *args, stream=st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            eng.score_device(pa, pb, n, ds.data_ptr(), de.data_ptr(), *args, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize(dev)
        out["ms"]["ungapped" if band is None else f"band{band}"] = e0.elapsed_time(e1) / reps
    eng.check_device_errors()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

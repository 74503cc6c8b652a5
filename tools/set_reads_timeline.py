"""ovl_set_reads at a config's read set (for rocprofv3 --kernel-trace --memory-copy-trace, OVL_TRACE_PIPE=1):
`reps` uploads with a 2 ms gap between calls on an engine per setting of OVL_READS_PACK2 (2-bit packed
upload, raw upload), interleaved; prints the median wall time per setting.

    python tools/set_reads_timeline.py [config] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.engine import encode_reads
    from ovlgraph.reads import config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    enc = encode_reads(reads)
    engines = {}
    for name, v in (("pack2", "1"), ("raw", "0")):
        os.environ["OVL_READS_PACK2"] = v
        engines[name] = OverlapEngine(0)
    os.environ.pop("OVL_READS_PACK2")
    times = {k: [] for k in engines}
    for _ in range(reps):
        for name, eng in engines.items():
            time.sleep(0.002)
            t0 = time.perf_counter()
            eng.set_reads(reads, enc)
            times[name].append((time.perf_counter() - t0) * 1e3)
            sys.stderr.write(f"== {name}\n")
    print({k: round(float(np.median(v)), 4) for k, v in times.items()})
    for eng in engines.values():
        eng.close()


if __name__ == "__main__":
    main()

"""ovl_set_reads of a read set that is already resident (same_reads: offsets compared, a digest of the bytes): the
cost a one-shot ovl_score_pairs call pays every call before scoring.  python tools/set_reads_probe.py [config]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "genome-assembly-using-overlap-graphs_amd"))


def main():
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.engine import encode_reads
    from ovlgraph.reads import config_reads
    cfg = sys.argv[1] if len(sys.argv) > 1 else "target"
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    enc = encode_reads(reads)
    eng = OverlapEngine(0)
    eng.set_reads(reads, enc)
    out = {"config": cfg, "reads_bytes": int(enc[0].nbytes)}
    for name, reps in (("warm", 20), ("timed", 200)):
        t0 = time.perf_counter()
        for _ in range(reps):
            eng.set_reads(reads, enc)
        out[name + "_ms"] = (time.perf_counter() - t0) / reps * 1e3
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Where the streamed cycle removal's time goes outside build_overlap_stream's own trace (OVL_TRACE_STREAM=1): the
target point's graph (GPU-scored), then remove_cycles_from_graph's lazy-graph steps one by one, timed.

    OVL_TRACE_STREAM=1 python tools/stream_probe.py [reps]
"""
import ctypes
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))


def main():
    import numpy as np
    from ovlgraph import _lib, overlapGraphs as og
    from ovlgraph.reads import config_reads
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    E = og.overlap_edges_k(config_reads("target", seed=0), 5)
    mod = og._digraph()
    for _ in range(reps):
        G = E.to_digraph()
        t = [time.perf_counter()]
        edges = G.__dict__["_ovl_edges"]
        off, heads, weights = edges.csr()
        t.append(time.perf_counter())
        names = edges.node_names()
        cnt = np.ascontiguousarray(edges.counts, dtype=np.int32)
        km = edges._keep_mask()
        tm = og._attr_template()
        fn = ctypes.cast(_lib.load().ovl_remove_cycles_stream, ctypes.c_void_p).value
        t.append(time.perf_counter())
        gc.disable()
        r = mod.build_overlap_stream(names, cnt, edges.a, edges.b, edges.score, edges.end, km, tm, fn,
                                     np.ascontiguousarray(off, dtype=np.int64),
                                     np.ascontiguousarray(heads, dtype=np.int32),
                                     np.ascontiguousarray(weights, dtype=np.int64))
        t.append(time.perf_counter())
        gc.enable()
        t.append(time.perf_counter())
        G._install(*r[:3])
        t.append(time.perf_counter())
        del r
        t.append(time.perf_counter())
        d = [round((b - a) * 1e3, 1) for a, b in zip(t, t[1:])]
        print(f"csr {d[0]} prep {d[1]} build_overlap_stream {d[2]} gc.enable {d[3]} install {d[4]} del {d[5]} ms",
              flush=True)
        del G, edges
        gc.collect()


if __name__ == "__main__":
    main()

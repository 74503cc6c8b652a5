"""Streamed cycle removal A/B: remove_cycles_from_graph on the target point's lazy graph through different builds of
the dict builder (build/replay_variants/<name>_digraph.so, and the tree's own), alternating, with OVL_TRACE_STREAM
lines on stderr; every variant must leave the same graph.  The columns are scored on the GPU, or, with --cpu, by
the oracle's closed form (tests-only checker, here only to make a graph on a machine without a GPU).

    python tools/stream_ab.py [rounds] [--cpu]
"""
import glob
import hashlib
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
import numpy as np  # noqa: E402

VAR = os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd", "build", "replay_variants")


def main():
    import gc
    from ovlgraph import overlapGraphs as og
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 3
    if "--cpu" in sys.argv:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        d, c = dedup_reads(config_reads("target", seed=0))
        a, b = enumerate_candidates(d, 5)
        s, e = oracle.batch_closed_form(d, a, b)
        edges = og.OverlapEdges(d, c, a, b, s, e)
    else:
        edges = og.overlap_edges_k(config_reads("target", seed=0), 5)
    mods = {"tree": None}
    for p in sorted(glob.glob(os.path.join(VAR, "*_digraph.so"))):
        spec = importlib.util.spec_from_file_location("ovlgraph._digraph", p)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        mods[os.path.basename(p)[:-len("_digraph.so")]] = m
    res = {k: [] for k in mods}
    sig = None
    for _ in range(rounds):
        for name, m in mods.items():
            og._digraph_mod = m
            G = edges.to_digraph()
            sys.stderr.write(f"== {name}\n")
            t0 = time.perf_counter()
            og.remove_cycles_from_graph(G)
            res[name].append(time.perf_counter() - t0)
            h = hashlib.sha1(repr((list(G.edges(data=True))[::97], [list(G.pred[v]) for v in list(G)[::53]])).encode()).hexdigest()
            assert sig is None or h == sig, name
            sig = h
            del G
            gc.collect()
    og._digraph_mod = None
    print(json.dumps({k: {"median": round(float(np.median(v)), 4), "all": [round(x, 4) for x in v]} for k, v in res.items()}))


if __name__ == "__main__":
    main()

"""Cycle-removal A/B on the box: the target point's overlap graph (scored on the GPU), then alternating runs of
replay variants (ovl_remove_cycles built from different sources into build/replay_variants/<name>.so) and of
the surviving-edge dict build (_digraph variants, build/replay_variants/<name>_digraph.so); every variant must
remove the same edges and build the same graph.

    python tools/replay_ab.py [rounds]
"""
import ctypes
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
    from ovlgraph.reads import config_reads
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    reads = config_reads("target", seed=0)
    edges = og.overlap_edges_k(reads, 5)
    off, heads, w = edges.csr()
    off = np.ascontiguousarray(off, np.int64)
    heads = np.ascontiguousarray(heads, np.int32)
    w = np.ascontiguousarray(w, np.int64)
    replays = {os.path.basename(p)[:-3]: ctypes.CDLL(p) for p in sorted(glob.glob(os.path.join(VAR, "*.so")))
               if not p.endswith("_digraph.so")}
    digraphs = {}
    for p in sorted(glob.glob(os.path.join(VAR, "*_digraph.so"))):
        spec = importlib.util.spec_from_file_location("ovlgraph._digraph", p)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        digraphs[os.path.basename(p)[:-len("_digraph.so")]] = m
    res = {"edges": int(heads.shape[0]), "replay_s": {k: [] for k in replays}, "dicts_s": {k: [] for k in digraphs}}
    ref = None
    alive = None
    for _ in range(rounds):
        for name, lib in replays.items():
            rem = np.zeros(heads.shape[0], np.int64)
            n = ctypes.c_int64(0)
            t0 = time.perf_counter()
            rc = lib.ovl_remove_cycles(off.ctypes.data_as(ctypes.c_void_p), heads.ctypes.data_as(ctypes.c_void_p),
                                       w.ctypes.data_as(ctypes.c_void_p), ctypes.c_int32(off.shape[0] - 1),
                                       rem.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n))
            res["replay_s"][name].append(time.perf_counter() - t0)
            got = rem[: n.value].copy()
            assert rc == 0
            if ref is None:
                ref = got
                alive = np.ones(heads.shape[0], np.uint8)
                alive[ref] = 0
            assert np.array_equal(got, ref), name
        sig = None
        for name, mod in digraphs.items():
            og._digraph_mod = mod
            G = edges.to_digraph()
            t0 = time.perf_counter()
            G._materialise(alive)
            res["dicts_s"][name].append(time.perf_counter() - t0)
            h = hashlib.sha1(repr((list(G.edges(data=True)), [list(G.pred[v]) for v in G])).encode()).hexdigest()
            assert sig is None or h == sig, name
            sig = h
            del G
            gc.collect()
    # the whole lazy-graph removal (what end_to_end times): replay then survivors' dicts, or both overlapped
    og._digraph_mod = None  # (the tree's own build)
    modes = ("serial", "stream_noscc", "stream")  # stream: with the component helper (OVL_STREAM_SCC)
    res["remove_cycles_s"] = {m: [] for m in modes}
    for _ in range(rounds):
        for mode in modes:
            og._STREAM_OFF = mode == "serial"
            os.environ["OVL_STREAM_SCC"] = "0" if mode == "stream_noscc" else "1"
            G = edges.to_digraph()
            t0 = time.perf_counter()
            og.remove_cycles_from_graph(G)
            res["remove_cycles_s"][mode].append(time.perf_counter() - t0)
            assert G.number_of_edges() == heads.shape[0] - ref.shape[0]
            del G
            gc.collect()
    res["remove_cycles_s"] = {m: {"median": round(float(np.median(v)), 4), "all": [round(x, 4) for x in v]}
                              for m, v in res["remove_cycles_s"].items()}
    res["removed"] = int(ref.shape[0])
    for k in ("replay_s", "dicts_s"):
        res[k] = {n: {"median": round(float(np.median(v)), 4), "min": round(float(np.min(v)), 4), "all": [round(x, 4) for x in v]}
                  for n, v in res[k].items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

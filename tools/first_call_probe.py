"""Why the first streamed removal of a process is slower than the next ones (bench.py end_to_end,
remove_cycles_runs_s): five calls on fresh lazy graphs of the target point, each call's stages, its page faults
(getrusage minor faults) and the process's resident size.

    python tools/first_call_probe.py
"""
import gc
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))


def rss_mb():
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20


def main():
    from ovlgraph import overlapGraphs as og
    from ovlgraph.reads import config_reads
    edges = og.overlap_edges_k(config_reads("target", seed=0), 5)
    out = {"edges": edges.n_edges(), "calls": []}
    for r in range(5):
        gc.collect()
        G = edges.to_digraph()
        t = {}
        f0 = resource.getrusage(resource.RUSAGE_SELF).ru_minflt
        m0 = rss_mb()
        t0 = time.perf_counter()
        og.remove_cycles_from_graph(G, timing=t)
        dt = time.perf_counter() - t0
        f1 = resource.getrusage(resource.RUSAGE_SELF).ru_minflt
        out["calls"].append({"s": round(dt, 4), "minor_faults": f1 - f0, "rss_before_mb": round(m0, 1),
                             "rss_after_mb": round(rss_mb(), 1),
                             "stages": {k: round(v, 4) for k, v in t.items() if isinstance(v, float)}})
        print(json.dumps(out["calls"][-1]), file=sys.stderr, flush=True)
        del G
    print(json.dumps(out))


if __name__ == "__main__":
    main()

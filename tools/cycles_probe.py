"""CPU probe: where remove_cycles_from_graph spends its time at a config's overlap graph.

The graph is built from the oracle's closed-form CPU scores (equal to the GPU's; no GPU needed), then
cycle removal runs with the stage split (CSR extraction, native replay, edge removal) timed.

    python tools/cycles_probe.py [config] [--check]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "genome-assembly-using-overlap-graphs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from ovlgraph import overlapGraphs as og  # noqa: E402
from ovlgraph.reads import config_reads  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "target"
    reads = config_reads(cfg, seed=0)
    t0 = time.perf_counter()
    G, _ = og.construct_overlap_graph_nx_k(reads, 5, scorer=lambda r, a, b: oracle.batch_closed_form(r, a, b),
                                           candidates="host")
    t1 = time.perf_counter()
    print(f"{cfg}: graph {G.number_of_nodes()} nodes {G.number_of_edges()} edges in {t1 - t0:.2f} s", flush=True)
    ref = None
    if "--check" in sys.argv:
        H = G.copy()
        og.remove_cycles_from_graph(H, native_edges=False)
        ref = list(H.edges())
    t2 = time.perf_counter()
    og.remove_cycles_from_graph(G, timing=(timing := {}))
    t3 = time.perf_counter()
    print(f"remove_cycles {t3 - t2:.2f} s: " + ", ".join(f"{k} {v:.3f} s" for k, v in timing.items()), flush=True)
    if ref is not None:
        print("identical to the per-edge path:", list(G.edges()) == ref)


if __name__ == "__main__":
    main()

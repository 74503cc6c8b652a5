"""Generate tests/golden/cycles.json from the reference's own remove_cycles_from_graph.

CONTAINER-ONLY, TEST INFRASTRUCTURE.  Run here (where /root/reference exists):

    python oracle/gen_golden_cycles.py

The reference module is imported exactly as oracle/gen_golden.py does (stub numba / Bio.Align
modules; ordinary ModuleNotFoundErrors, not permission denials).  remove_cycles_from_graph
(overlapGraphs.py:106-130) is pure networkx, so no scoring typing is involved.  Each record holds
the input graph (node order, out-edges in adjacency order with their weights) and the edges the
reference leaves, in G.edges order.  No reference source is copied.

Inputs: random digraphs (dense and sparse, self-loops, tied and negative weights, shuffled node
order) and overlap graphs of PhiX reads built by this package's host path (identical to the
reference's builder, tests/test_graph_assembly_cpu.py).
"""
from __future__ import annotations

import json
import os
import random
import sys
import time

import networkx as nx

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import GOLDEN, import_reference  # noqa: E402


def graph_record(G, name):
    nodes = list(G)
    return {"name": name, "nodes": nodes,
            "adj": [[[v, d["weight"]] for v, d in G._adj[u].items()] for u in nodes]}


def rebuild(rec):
    G = nx.DiGraph()
    G.add_nodes_from(rec["nodes"])
    for u, nbrs in zip(rec["nodes"], rec["adj"]):
        for v, w in nbrs:
            G.add_edge(u, v, weight=w)
    return G


def random_graph(rng, n, p, loops=0.1, wlo=-3, whi=5):
    G = nx.DiGraph()
    order = list(range(n))
    rng.shuffle(order)
    G.add_nodes_from(order)
    edges = [(u, v) for u in range(n) for v in range(n) if (u != v or rng.random() < loops) and rng.random() < p]
    rng.shuffle(edges)
    for u, v in edges:
        G.add_edge(u, v, weight=rng.randint(wlo, whi))
    return G


def overlap_graph(n_reads, seed):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "genome-assembly-using-overlap-graphs_amd"))
    import oracle
    from ovlgraph import overlapGraphs as og
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    oracle.build()
    reads, copies = dedup_reads(simulate_reads(read_genome_from_fasta(), 100, n_reads, 0.01, seed=seed))
    a, b = enumerate_candidates(reads, 5)
    sc, en = oracle.batch_ungapped(reads, a, b, 10, -1)
    G = og.assemble_graph(reads, copies, a, b, sc, en)
    # node names are read strings: index them to keep the fixture small
    names = {v: i for i, v in enumerate(G)}
    H = nx.DiGraph()
    H.add_nodes_from(range(len(names)))
    for u, v, d in G.edges(data=True):
        H.add_edge(names[u], names[v], weight=d["weight"])
    return H


def assembly_cases(aligners, overlapGraphs, gefr):
    """assemble_contigs_using_overlap_graphs end to end on small read sets (scoring typed as Numba does,
    as in gen_golden.py)."""
    import contextlib
    import functools
    import io
    import numpy as np
    from gen_golden import REF
    overlapGraphs.overlap_alignment = functools.partial(aligners.overlap_alignment, indel=np.int64(-(2 ** 31)))
    genome = gefr.read_genome_from_fasta(os.path.join(REF, "sequence.fasta"))
    rng = random.Random(7)
    cases = []
    for n_reads, l, p, k in ((120, 100, 0.0, 5), (200, 80, 0.01, 5), (150, 60, 0.02, 3)):
        reads = []
        for _ in range(n_reads):
            st = rng.randrange(len(genome))
            r = genome[st:st + l]
            r = "".join(rng.choice([c for c in "ACGT" if c != ch]) if rng.random() < p else ch for ch in r)
            reads.append(r)
        reads += reads[:3]  # copies
        params = {"N": len(reads), "l": l, "k": k, "error_prob": p, "experiment_name": "golden", "num_iteration": 0}
        t0 = time.time()
        with contextlib.redirect_stdout(io.StringIO()):
            contigs = overlapGraphs.assemble_contigs_using_overlap_graphs(reads, k=k, params=params)
        cases.append({"reads": reads, "k": k, "params": params, "contigs": list(contigs),
                      "reference_seconds": round(time.time() - t0, 2)})
        print("assembly", n_reads, l, p, k, len(contigs), "contigs", f"{time.time() - t0:.1f} s", flush=True)
    return cases


def main():
    aligners, overlapGraphs, gefr = import_reference()
    rng = random.Random(20261016)
    inputs = []
    for i in range(60):
        n = rng.randint(1, 40)
        inputs.append((random_graph(rng, n, rng.choice([0.03, 0.08, 0.15, 0.3, 0.6])), f"random{i}"))
    for i in range(6):
        inputs.append((random_graph(rng, rng.randint(60, 120), rng.choice([0.02, 0.05]), wlo=0, whi=2),
                       f"random_ties{i}"))
    for n_reads, seed in ((300, 1), (800, 2), (1500, 3)):
        inputs.append((overlap_graph(n_reads, seed), f"phix_l100_n{n_reads}"))
    records = []
    for G, name in inputs:
        rec = graph_record(G, name)
        t0 = time.time()
        H = overlapGraphs.remove_cycles_from_graph(rebuild(rec))
        rec["kept"] = [[u, v] for u, v in H.edges()]
        rec["removed"] = G.number_of_edges() - H.number_of_edges()
        rec["reference_seconds"] = round(time.time() - t0, 3)
        records.append(rec)
        print(name, G.number_of_nodes(), G.number_of_edges(), "removed", rec["removed"],
              f"{rec['reference_seconds']} s", flush=True)
    with open(os.path.join(GOLDEN, "cycles.json"), "w") as fh:
        json.dump({"source": "reference overlapGraphs.remove_cycles_from_graph (networkx "
                             f"{nx.__version__})", "records": records}, fh, separators=(",", ":"))
    with open(os.path.join(GOLDEN, "assembly.json"), "w") as fh:
        json.dump({"source": "reference overlapGraphs.assemble_contigs_using_overlap_graphs (numba absent: njit "
                             "identity, scoring args as np.int64)",
                   "cases": assembly_cases(aligners, overlapGraphs, gefr)}, fh, separators=(",", ":"))


if __name__ == "__main__":
    main()

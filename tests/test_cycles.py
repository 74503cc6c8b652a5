"""remove_cycles_from_graph (overlapGraphs.py:106-130): the native exact replay (csrc/ovl_graph.cpp,
ovl_remove_cycles; host code, no GPU) removes exactly the reference's edges.

Pinned by tests/golden/cycles.json, written by oracle/gen_golden_cycles.py from the reference's own
function; the oracle's restatement (the same networkx loop) is checked against those records too and
then used for larger random graphs and PhiX overlap graphs.
"""
import random

import networkx as nx
import numpy as np
import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def golden_cycles():
    return load_golden("cycles.json")["records"]


def _rebuild(rec):
    G = nx.DiGraph()
    G.add_nodes_from(rec["nodes"])
    for u, nbrs in zip(rec["nodes"], rec["adj"]):
        for v, w in nbrs:
            G.add_edge(u, v, weight=w)
    return G


def _same(G1, G2):
    return (list(G1.nodes()) == list(G2.nodes()) and list(G1.edges(data=True)) == list(G2.edges(data=True))
            and all(list(G1.pred[n]) == list(G2.pred[n]) for n in G1))


def test_native_matches_reference_golden(golden_cycles):
    from ovlgraph.overlapGraphs import remove_cycles_from_graph
    assert len(golden_cycles) >= 60
    for rec in golden_cycles:
        G = remove_cycles_from_graph(_rebuild(rec))
        assert [[u, v] for u, v in G.edges()] == rec["kept"], rec["name"]
        assert nx.is_directed_acyclic_graph(G)


def test_oracle_matches_reference_golden(oracle_mod, golden_cycles):
    for rec in golden_cycles:
        if rec["reference_seconds"] > 0.5:
            continue
        G = oracle_mod.remove_cycles(_rebuild(rec))
        assert [[u, v] for u, v in G.edges()] == rec["kept"], rec["name"]


def _random_graph(rng, n, p, loops=0.1, wlo=-3, whi=5):
    G = nx.DiGraph()
    order = list(range(n))
    rng.shuffle(order)
    G.add_nodes_from(order)
    edges = [(u, v) for u in range(n) for v in range(n) if (u != v or rng.random() < loops) and rng.random() < p]
    rng.shuffle(edges)
    for u, v in edges:
        G.add_edge(u, v, weight=rng.randint(wlo, whi), end_position=u)
    return G


@pytest.mark.parametrize("seed", range(6))
def test_native_matches_oracle_random(oracle_mod, seed):
    from ovlgraph.overlapGraphs import remove_cycles_from_graph
    rng = random.Random(seed)
    for _ in range(40):
        G = _random_graph(rng, rng.randint(1, 60), rng.choice([0.02, 0.05, 0.1, 0.3, 0.6]),
                          whi=rng.choice([0, 1, 5, 1000]))
        assert _same(oracle_mod.remove_cycles(G.copy()), remove_cycles_from_graph(G.copy()))


@pytest.mark.parametrize("seed", range(3))
def test_native_matches_oracle_wide_weights(oracle_mod, seed):
    """Weights beyond int32 (the replay's 16-byte edge records; int32 weights take the 12-byte ones): ties
    and order among weights that differ only above bit 31 or only below it."""
    from ovlgraph.overlapGraphs import remove_cycles_from_graph
    rng = random.Random(100 + seed)
    for _ in range(30):
        G = _random_graph(rng, rng.randint(2, 40), rng.choice([0.05, 0.1, 0.3]), whi=3)
        for u, v, d in G.edges(data=True):
            d["weight"] = rng.choice([-1, 0, 1, 2]) * (1 << 33) + d["weight"]
        assert _same(oracle_mod.remove_cycles(G.copy()), remove_cycles_from_graph(G.copy()))


def _layered_graph(rng, blobs):
    """Strongly connected blobs joined by DAG edges, acyclic tails in and out of them, node order
    shuffled: starts that reach only acyclic territory, DFS excursions into nodes that can no longer
    reach a cycle (the native replay's settled nodes) and blobs that break up as edges go."""
    G = nx.DiGraph()
    nodes, groups = [], []
    for bi in range(blobs):
        size = rng.randint(1, 9)
        grp = [f"b{bi}_{i}" for i in range(size)]
        groups.append(grp)
        nodes += grp
    tails = [f"t{i}" for i in range(rng.randint(0, 25))]
    order = nodes + tails
    rng.shuffle(order)
    G.add_nodes_from(order)
    edges = []
    for grp in groups:
        for u in grp:
            for v in grp:
                if (u != v or rng.random() < 0.05) and rng.random() < 0.5:
                    edges.append((u, v))
    for i in range(len(groups)):
        for j in range(i + 1, len(groups)):
            if rng.random() < 0.3:
                edges.append((rng.choice(groups[i]), rng.choice(groups[j])))
    rank = {t: i for i, t in enumerate(tails)}
    for t in tails:
        for _ in range(rng.randint(1, 4)):
            x = rng.choice(nodes + tails)
            if x in rank and rank[x] <= rank[t]:
                continue
            edges.append((t, x) if rng.random() < 0.5 or x in rank else (x, t))
    rng.shuffle(edges)
    for u, v in edges:
        G.add_edge(u, v, weight=rng.randint(-2, 6))
    return G


@pytest.mark.parametrize("settle", ["default", "0"])
def test_native_matches_oracle_layered(oracle_mod, monkeypatch, settle):
    """Settled-node skipping (ovl_graph.cpp): with the settled set kept exact after every removal (the
    default) and with no settled-node pruning at all, the replay must remove the oracle's edges."""
    from ovlgraph.overlapGraphs import remove_cycles_from_graph
    if settle != "default":
        monkeypatch.setenv("OVL_CYCLES_SETTLE", settle)
    rng = random.Random(1234)
    for _ in range(60):
        G = _layered_graph(rng, rng.randint(1, 8))
        assert _same(oracle_mod.remove_cycles(G.copy()), remove_cycles_from_graph(G.copy()))
    for _ in range(20):
        G = _random_graph(rng, rng.randint(1, 40), rng.choice([0.03, 0.08, 0.2]), whi=rng.choice([1, 5]))
        assert _same(oracle_mod.remove_cycles(G.copy()), remove_cycles_from_graph(G.copy()))


def test_native_matches_oracle_overlap_graph(oracle_mod):
    """A PhiX overlap graph (1,200 reads, l = 100, p = 0.01, k = 5) with its copies and attributes."""
    from ovlgraph import overlapGraphs as og
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    reads, copies = dedup_reads(simulate_reads(read_genome_from_fasta(), 100, 1200, 0.01, seed=9))
    a, b = enumerate_candidates(reads, 5)
    sc, en = oracle_mod.batch_ungapped(reads, a, b, 10, -1)
    G = og.assemble_graph(reads, copies, a, b, sc, en)
    H = og.remove_cycles_from_graph(G.copy())
    assert H.number_of_edges() < G.number_of_edges()
    assert _same(oracle_mod.remove_cycles(G.copy()), H)


def test_degenerate_graphs_and_errors():
    from ovlgraph.overlapGraphs import remove_cycles_from_graph
    assert remove_cycles_from_graph(nx.DiGraph()).number_of_nodes() == 0
    G = nx.DiGraph()
    G.add_nodes_from("abc")
    assert list(remove_cycles_from_graph(G).nodes()) == ["a", "b", "c"]
    G.add_edge("a", "a", weight=3)
    assert remove_cycles_from_graph(G).number_of_edges() == 0
    G.add_edge("a", "b", weight=1.5)
    G.add_edge("b", "a", weight=2)
    with pytest.raises(TypeError):
        remove_cycles_from_graph(G)


def test_abi_rejects_bad_csr():
    import ctypes
    from ovlgraph import _lib
    L = _lib.load()
    off = np.array([0, 2, 1], dtype=np.int64)  # decreasing offsets
    head = np.array([1, 0], dtype=np.int32)
    w = np.array([1, 1], dtype=np.int64)
    rem = np.zeros(2, dtype=np.int64)
    n = ctypes.c_int64()
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    assert L.ovl_remove_cycles(p(off), p(head), p(w), 2, p(rem), ctypes.byref(n)) == -1  # OVL_E_ARG
    off = np.array([0, 1, 2], dtype=np.int64)
    head = np.array([1, 5], dtype=np.int32)  # head out of range
    assert L.ovl_remove_cycles(p(off), p(head), p(w), 2, p(rem), ctypes.byref(n)) < 0
    head = np.array([1, 0], dtype=np.int32)
    assert L.ovl_remove_cycles(p(off), p(head), p(w), 2, p(rem), ctypes.byref(n)) == 0 and n.value == 1


@pytest.mark.parametrize("seed", range(4))
def test_native_edge_passes_match_python_passes(seed):
    """The C passes around the replay (csr + bulk remove_edges, csrc/ovl_digraph.c) leave the same graph
    as the Python passes (generators + remove_edge per edge): nodes, successor/predecessor order, data."""
    from ovlgraph import overlapGraphs as og
    if og._digraph() is None:
        pytest.skip("ovlgraph._digraph not built")
    rng = random.Random(100 + seed)
    for _ in range(25):
        G = (_layered_graph(rng, rng.randint(1, 8)) if rng.random() < 0.5 else
             _random_graph(rng, rng.randint(1, 50), rng.choice([0.05, 0.2, 0.5]), whi=rng.choice([1, 5, 1000])))
        if G.number_of_edges() and rng.random() < 0.3:  # numpy integer weights are accepted by both
            u, v = next(iter(G.edges()))
            G[u][v]["weight"] = np.int64(G[u][v]["weight"])
        t_native, t_py = {}, {}
        H1 = og.remove_cycles_from_graph(G.copy(), native_edges=True, timing=t_native)
        H2 = og.remove_cycles_from_graph(G.copy(), native_edges=False, timing=t_py)
        assert _same(H1, H2) and t_native["removed"] == t_py["removed"]
        assert all(list(H1.pred[n]) == list(H2.pred[n]) for n in H1)
        assert nx.is_directed_acyclic_graph(H1)


def test_native_edge_passes_errors_and_fallback():
    from ovlgraph import overlapGraphs as og
    if og._digraph() is None:
        pytest.skip("ovlgraph._digraph not built")
    for bad in (1.5, True, np.bool_(True), "3", None):
        G = nx.DiGraph()
        G.add_edge("a", "b", weight=2)
        G.add_edge("b", "a", weight=bad)
        with pytest.raises(TypeError):
            og.remove_cycles_from_graph(G, native_edges=True)
    G = nx.DiGraph()
    G.add_edge("a", "b", weight=2)
    G.add_edge("b", "a", end_position=1)
    with pytest.raises(KeyError):
        og.remove_cycles_from_graph(G, native_edges=True)

    class Sub(nx.DiGraph):  # a DiGraph subclass keeps networkx's own remove_edge (Python passes)
        pass
    rng = random.Random(7)
    G = _random_graph(rng, 30, 0.2)
    S = Sub(G)
    H = og.remove_cycles_from_graph(S)
    assert type(H) is Sub and _same(H, og.remove_cycles_from_graph(G.copy(), native_edges=False))
    mod = og._digraph()
    assert mod.csr(list(G), {n: dict(G._adj[n]) for n in G}) is not None
    from collections import OrderedDict
    assert mod.csr(list(G), {n: OrderedDict(G._adj[n]) for n in G}) is None
    E = nx.DiGraph()
    E.add_edge("a", "b", weight=1)
    with pytest.raises(KeyError):  # b -> a is not an edge
        mod.remove_edges(E._succ, E._pred, ["a", "b"], np.array([1], np.int64), np.array([0], np.int64))
    mod.remove_edges(E._succ, E._pred, ["a", "b"], np.array([0], np.int64), np.array([1], np.int64))
    assert E.number_of_edges() == 0 and list(E.pred["b"]) == []

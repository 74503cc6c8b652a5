"""Graph assembly order/attributes of the drop-in builders, with oracle scores injected (no GPU).

The product builders call the GPU engine; here the same code path is fed the
oracle's (score, end) through the `scorer` hook to check node order, edge
order, copies and attribute types against the reference's golden graphs.
"""
import contextlib
import io

import pytest

from conftest import assert_graph_matches_record
from ovlgraph import overlapGraphs as og


def _oracle_scorer(oracle_mod):
    return lambda reads, a, b: oracle_mod.batch_dp(reads, a, b)


def test_nx_k_graphs_match_golden(golden_graphs, oracle_mod):
    for rec in golden_graphs["graphs"]:
        copies = None
        if rec["fn"] == "construct_overlap_graph_nx_k":
            G, copies = og.construct_overlap_graph_nx_k(rec["reads"], scorer=_oracle_scorer(oracle_mod),
                                                        **rec["kwargs"])
        elif rec["fn"] == "construct_overlap_graph_string":
            G, copies = og.construct_overlap_graph_string(rec["reads"], scorer=_oracle_scorer(oracle_mod))
        else:
            with contextlib.redirect_stdout(io.StringIO()):
                G = og.construct_string_graph(rec["reads"], scorer=_oracle_scorer(oracle_mod))
        assert_graph_matches_record(G, rec, copies)


def test_alias():
    assert og.build_overlap_graph is og.construct_overlap_graph_nx_k


def test_assert_k_nonnegative():
    import pytest
    with pytest.raises(AssertionError):
        og.construct_overlap_graph_nx_k(["ACGT"], k=-1)


def test_no_candidates_needs_no_gpu():
    # host enumeration finds no pair -> nothing is scored -> no device needed
    G, copies = og.construct_overlap_graph_nx_k(["AAAA", "CCCC", "AAAA"], k=2, candidates="host")
    assert list(G.nodes()) == ["AAAA_0", "AAAA_1", "CCCC_0"]
    assert G.number_of_edges() == 0 and copies == {"AAAA": 2, "CCCC": 1}


def _same_graph(G1, G2):
    assert list(G1.nodes()) == list(G2.nodes())
    assert list(G1.edges(data=True)) == list(G2.edges(data=True))
    for n in G1.nodes():
        assert list(G1.successors(n)) == list(G2.successors(n))
        assert list(G1.predecessors(n)) == list(G2.predecessors(n))
        for v in G2.successors(n):
            assert G2[n][v] is G2.pred[v][n]  # one attribute dict per edge, as add_edge shares it
            assert type(G2[n][v]["weight"]) is int and type(G2[n][v]["end_position"]) is int


def _scored_case(seed, n_reads=300, alphabet="ACG", k=2):
    import random

    import numpy as np
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    rng = random.Random(seed)
    reads = ["".join(rng.choice(alphabet) for _ in range(rng.randint(1, 6))) for _ in range(n_reads)]
    d, c = dedup_reads(reads)
    a, b = enumerate_candidates(d, k)
    sc = np.array([rng.randint(-3, 9) for _ in range(len(a))], np.int32)
    en = np.arange(len(a), dtype=np.int32)
    return d, c, a, b, sc, en


@pytest.mark.parametrize("native", [True, False])
def test_direct_assembly_matches_networkx_construction(native):
    """assemble_graph_direct builds the same DiGraph as networkx's add_edges_from (copies, filters, empty),
    through the C builder (csrc/ovl_digraph.c) and through the Python grouping."""
    import numpy as np
    for seed in (1, 2, 3):
        d, c, a, b, sc, en = _scored_case(seed)
        assert max(c) > 1  # copies exercised
        for ms in (None, 0, 5):
            _same_graph(og.assemble_graph(d, c, a, b, sc, en, ms),
                        og.assemble_graph_direct(d, c, a, b, sc, en, ms, native=native))
    z = np.zeros(0, np.int32)
    _same_graph(og.assemble_graph(["A"], [2], z, z, z, z), og.assemble_graph_direct(["A"], [2], z, z, z, z, native=native))
    _same_graph(og.assemble_graph([], [], z, z, z, z), og.assemble_graph_direct([], [], z, z, z, z, native=native))


def test_native_builder_attribute_dicts_behave_like_dicts():
    """The C builder's per-edge dicts share one key table (PEP 412) but are ordinary, independent dicts."""
    import copy
    import pickle
    d, c, a, b, sc, en = _scored_case(4)
    G = og.assemble_graph_direct(d, c, a, b, sc, en, native=True)
    (u1, v1, d1), (u2, v2, d2) = list(G.edges(data=True))[:2]
    assert type(d1) is dict and d1 is G.pred[v1][u1]
    d1["color"] = "red"
    d1["weight"] += 1000
    assert "color" not in d2 and d2["weight"] < 1000
    del d1["end_position"]
    assert list(d1) == ["weight", "color"] and list(d2) == ["weight", "end_position"]
    H = pickle.loads(pickle.dumps(G))
    assert list(H.edges(data=True)) == list(G.edges(data=True))
    assert list(copy.deepcopy(G).edges(data=True)) == list(G.edges(data=True))
    G.add_edge(u2, v2, weight=-1)  # networkx updates the existing dict in place
    assert G[u2][v2] is d2 and d2 == {"weight": -1, "end_position": int(d2["end_position"])}


def test_overlap_edges_columns_match_graph():
    import numpy as np
    d, c, a, b, sc, en = _scored_case(7)
    for ms in (None, 0):
        E = og.OverlapEdges(d, c, a, b, sc, en, min_score=ms)
        G = E.to_digraph()
        names = E.node_names()
        u, v, w, e = E.edge_arrays()
        assert E.n_edges() == G.number_of_edges() == u.shape[0]
        # edge_arrays are in global insertion order; the graph iterates per source node,
        # i.e. the same edges stably grouped by u
        o = np.argsort(u, kind="stable")
        assert [(names[x], names[y], {"weight": int(s), "end_position": int(t)})
                for x, y, s, t in zip(u[o], v[o], w[o], e[o])] == list(G.edges(data=True))
        # and per target node the insertion order is the predecessor order
        for node in range(0, len(names), 7):
            assert [names[x] for x in u[v == node]] == list(G.predecessors(names[node]))
        assert E.read_copies() == dict(zip(d, c))


def test_overlap_edges_k_golden_graphs(golden_graphs, oracle_mod):
    for rec in golden_graphs["graphs"]:
        if rec["fn"] != "construct_overlap_graph_nx_k":
            continue
        E = og.overlap_edges_k(rec["reads"], scorer=_oracle_scorer(oracle_mod), **rec["kwargs"])
        assert_graph_matches_record(E.to_digraph(), rec, E.read_copies())


def test_assembly_pipeline_matches_reference_contigs(oracle_mod):
    """assemble_contigs_using_overlap_graphs (overlapGraphs.py:151-193): graph, native cycle removal,
    topological order and contig walks give the reference's contigs (tests/golden/assembly.json,
    written by oracle/gen_golden_cycles.py from the reference function), with oracle scores."""
    from conftest import load_golden
    cases = load_golden("assembly.json")["cases"]
    assert len(cases) == 3
    for case in cases:
        out = io.StringIO()
        with contextlib.redirect_stdout(out):
            contigs = og.assemble_contigs_using_overlap_graphs(case["reads"], k=case["k"], params=case["params"],
                                                               scorer=_oracle_scorer(oracle_mod))
        assert contigs == case["contigs"]
        assert "Removing cycles from graph for experiment_name=golden" in out.getvalue()

"""Graph assembly order/attributes of the drop-in builders, with oracle scores injected (no GPU).

The product builders call the GPU engine; here the same code path is fed the
oracle's (score, end) through the `scorer` hook to check node order, edge
order, copies and attribute types against the reference's golden graphs.
"""
import contextlib
import io

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

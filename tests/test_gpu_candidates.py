"""Device k-mer candidate enumeration (ovl_candidates) vs the host restatement, bit-exact.

``candidates.enumerate_candidates`` is itself pinned to the literal loop
restatement of overlapGraphs.py:30-52 by tests/test_candidates.py (CPU) and to
the reference's graphs by the golden fixtures; here the device list must be
identical element for element (same pairs, same order).
"""
import random

import numpy as np
import pytest

from conftest import assert_graph_matches_record

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from ovlgraph import OverlapEngine
    eng = OverlapEngine(0)
    yield eng
    eng.close()


def _check(engine, distinct, k):
    from ovlgraph.candidates import enumerate_candidates
    engine.set_reads(distinct)
    a, b = engine.candidates(k)
    ra, rb = enumerate_candidates(distinct, k)
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(b, rb)
    return a.shape[0]


def _distinct(reads):
    from ovlgraph.candidates import dedup_reads
    return dedup_reads(reads)[0]


@pytest.mark.parametrize("k", [0, 1, 2, 3, 5, 8, 10, 15, 29])
def test_random_reads_all_k(engine, k):
    rng = random.Random(100 + k)
    # a small alphabet window so many prefixes/suffixes collide; lengths around k
    reads = ["".join(rng.choice("ACGT") for _ in range(rng.randint(0, 40))) for _ in range(700)]
    reads += ["A" * rng.randint(1, 12) for _ in range(30)]  # homopolymers: self-matching keys
    distinct = _distinct(reads)
    if k == 0:
        distinct = distinct[:300]
    _check(engine, distinct, k)


@pytest.mark.parametrize("cfg", ["cfg1", "cfg2", "target"])
def test_config_candidate_lists(engine, cfg):
    from ovlgraph.reads import config_reads
    distinct = _distinct(config_reads(cfg))
    n = _check(engine, distinct, 5)
    assert n > 0


@pytest.mark.parametrize("k", [5, 10, 15])
def test_simulated_reads_other_k(engine, k):
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    distinct = _distinct(simulate_reads(read_genome_from_fasta(), 100, 5000, 0.01, seed=k))
    _check(engine, distinct, k)


@pytest.mark.parametrize("alphabet,k", [("ACGTN", 5), ("ACGTNacgt", 14), ("ACGTNRYKMSWBDHV-xyz", 7)])
def test_wider_alphabets(engine, alphabet, k):
    rng = random.Random(len(alphabet))
    reads = ["".join(rng.choice(alphabet[:4] if rng.random() < 0.7 else alphabet) for _ in range(rng.randint(1, 30)))
             for _ in range(500)]
    _check(engine, _distinct(reads), k)


def test_key_limits(engine):
    from ovlgraph import OvlError
    engine.set_reads(["ACGT", "CGTA"])
    assert engine.candidates(29)[0].shape[0] == 0
    with pytest.raises(OvlError, match="OVL_E_UNSUPPORTED"):
        engine.candidates(30)
    with pytest.raises(AssertionError):
        engine.candidates(-1)


def test_edge_cases(engine):
    for distinct, k in ((["A"], 5), ([""], 3), (["", "A", "AA"], 1), (["AC", "CA", "ACA", "CAC"], 1),
                        (["ACGT"] + ["T" + "ACGT"[i:] for i in range(4)], 2)):
        _check(engine, distinct, k)
    engine.set_reads([])
    a, b = engine.candidates(5)
    assert a.shape[0] == 0


def test_resident_candidates_scored_like_host_pairs(engine, oracle_mod):
    from ovlgraph.reads import config_reads
    distinct = _distinct(config_reads("cfg2"))
    engine.set_reads(distinct)
    a, b = engine.candidates(5)
    sc, en = engine.score_candidates()
    rs, re_ = oracle_mod.batch_ungapped(distinct, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)
    hs, he = engine.score(a, b)
    np.testing.assert_array_equal(sc, hs)
    np.testing.assert_array_equal(en, he)


@pytest.mark.parametrize("mode", ["device", "host"])
def test_golden_graphs_both_candidate_paths(engine, golden_graphs, mode):
    from ovlgraph import overlapGraphs as og
    for rec in golden_graphs["graphs"]:
        if rec["fn"] != "construct_overlap_graph_nx_k":
            continue
        G, copies = og.construct_overlap_graph_nx_k(rec["reads"], engine=engine, candidates=mode, **rec["kwargs"])
        assert_graph_matches_record(G, rec, copies)


def test_cfg4_full_pipeline_vs_oracle(engine, oracle_mod):
    """Config 4 (random 1 Mbp genome, 200k reads, ~38 M pairs): device enumeration == host
    enumeration, and every resident candidate scored == the oracle."""
    from ovlgraph.candidates import enumerate_candidates
    from ovlgraph.reads import config_reads
    distinct = _distinct(config_reads("cfg4"))
    engine.set_reads(distinct)
    a, b = engine.candidates(5)
    ra, rb = enumerate_candidates(distinct, 5)
    np.testing.assert_array_equal(a, ra)
    np.testing.assert_array_equal(b, rb)
    assert a.shape[0] > 30_000_000
    sc, en = engine.score_candidates()
    rs, re_ = oracle_mod.batch_ungapped(distinct, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)

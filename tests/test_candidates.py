"""Host-side candidate enumeration and read simulation (no GPU)."""
import random

import numpy as np
import pytest


from ovlgraph.candidates import dedup_reads, enumerate_candidates, enumerate_candidates_loop
from ovlgraph.reads import CONFIGS, read_genome_from_fasta, simulate_reads


def _rand_reads(rng, n, lmin, lmax, alphabet="ACGT"):
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(lmin, lmax))) for _ in range(n)]


@pytest.mark.parametrize("k", [0, 1, 2, 3, 5, 10])
def test_vectorised_matches_loop(k):
    rng = random.Random(k)
    reads = _rand_reads(rng, 150, 1, 12, "ACG")
    reads += reads[:20]  # duplicates
    distinct, counts = dedup_reads(reads)
    a1, b1 = enumerate_candidates(distinct, k)
    a2, b2 = enumerate_candidates_loop(distinct, k)
    assert a1.tolist() == a2.tolist()
    assert b1.tolist() == b2.tolist()


def test_dedup_order_and_counts():
    d, c = dedup_reads(["B", "A", "B", "C", "A", "B"])
    assert d == ["B", "A", "C"] and c == [3, 2, 1]


def test_negative_k_asserts():
    with pytest.raises(AssertionError):
        enumerate_candidates(["ACGT"], -1)


def test_empty():
    a, b = enumerate_candidates([], 5)
    assert a.size == 0 and b.size == 0


def test_enumeration_reproduces_golden_edge_order(golden_graphs):
    for rec in golden_graphs["graphs"]:
        if rec["fn"] != "construct_overlap_graph_nx_k":
            continue
        distinct, counts = dedup_reads(rec["reads"])
        assert distinct == rec["distinct"]
        a, b = enumerate_candidates(distinct, rec["kwargs"]["k"])
        # G.edges() is adjacency order: per source node, successors in insertion order.
        # From copy 0 of each read, the successor reads (copies collapsed) must be
        # exactly that read's candidates in enumeration order.
        succ = {}
        for ia, ca, ib, cb, w, e in rec["edges"]:
            if ca == 0:
                lst = succ.setdefault(ia, [])
                if not lst or lst[-1] != ib:
                    lst.append(ib)
        cand = {}
        for x, y in zip(a.tolist(), b.tolist()):
            cand.setdefault(x, []).append(y)
        assert succ == cand


def test_phix_genome():
    g = read_genome_from_fasta()
    assert len(g) == 5386 and set(g) == set("ACGT")


def test_simulator_properties():
    g = read_genome_from_fasta()
    reads = simulate_reads(g, 100, 4000, 0.0, seed=3)
    assert all(1 <= len(r) <= 100 for r in reads)
    short = [r for r in reads if len(r) < 100]
    assert all(g.endswith(r) for r in short)  # truncated at the genome end, never cyclic
    assert all(r in g for r in reads[:200])
    err = simulate_reads(g, 100, 2000, 0.05, seed=3)
    clean = simulate_reads(g, 100, 2000, 0.0, seed=3)
    # same starts (same seed stream for starts), substitutions only
    diffs = sum(x != y for r1, r2 in zip(err, clean) for x, y in zip(r1, r2))
    total = sum(len(r) for r in clean)
    assert 0.03 < diffs / total < 0.07
    assert simulate_reads(g, 100, 50, 0.01, seed=9) == simulate_reads(g, 100, 50, 0.01, seed=9)


def test_config_table():
    assert CONFIGS["cfg2"] == dict(genome="phix", N=10_000, l=100, p=0.01, k=5)

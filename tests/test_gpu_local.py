"""GPU local_alignment (aligners.py:85-167) vs the reference's golden outputs and the oracle, bit-exact.

The kernel runs one pair on many wavefronts (64-row strips handed over through L2), so
the larger cases here are what exercise the cross-CU hand-off: several strips, several
64-column chunks, uneven progress between producer and consumer.
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from ovlgraph import OverlapEngine
    eng = OverlapEngine(0)
    yield eng
    eng.close()


def test_local_alignment_golden(engine):
    from conftest import load_golden
    from ovlgraph import aligners
    d = load_golden("local_alignment.json")
    for rec in d["pairs"]:
        got = aligners.local_alignment(rec["query"], rec["reference"], rec["match"], rec["mismatch"], rec["indel"],
                                       engine=engine)
        assert got == (rec["to_print"], rec["aligned_reference"], rec["aligned_query"], rec["score"], rec["start"],
                       rec["end"]), rec["query"][:30]
    for rec in d["align_to_reference"]:
        got = aligners.align_read_or_contig_to_reference(rec["item"], rec["reference"], rec["read_length"],
                                                         engine=engine)
        assert got == (rec["to_print"], rec["aligned_reference"], rec["aligned_query"], rec["score"], rec["start"],
                       rec["end"])


def _genome_pair(rng, genome, n, m, p_sub=0.02, p_indel=0.01):
    st = rng.randint(0, len(genome) - m)
    ref = genome[st:st + m]
    o = rng.randint(0, max(0, m - n))
    out = []
    for ch in ref[o:o + n]:
        u = rng.random()
        if u < p_indel / 2:
            continue
        if u < p_indel:
            out.append(rng.choice("ACGT"))
        out.append(rng.choice("ACGT") if rng.random() < p_sub else ch)
    return "".join(out), ref


@pytest.mark.parametrize("n,m", [(1, 1), (63, 64), (64, 65), (65, 63), (130, 1000), (700, 129), (1000, 3000)])
def test_local_vs_oracle_sizes(engine, oracle_mod, n, m):
    from ovlgraph import aligners
    from ovlgraph.reads import read_genome_from_fasta
    rng = random.Random(n * 7 + m)
    genome = read_genome_from_fasta()
    q, r = _genome_pair(rng, genome, n, m)
    for params in ((10, -1, -1), (2, -3, -5), (1, -1, -1)):
        got = aligners.local_alignment(q, r, *params, engine=engine)
        exp = oracle_mod.local_alignment(q, r, *params)
        assert got == exp, (n, m, params)


def test_local_unrelated_and_score_only(engine, oracle_mod):
    rng = random.Random(3)
    for _ in range(10):
        q = "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 300)))
        r = "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 300)))
        sc, ei, ej, si, sj, ops = engine.local_align(q, r, traceback=False)
        _, _, _, esc, _, eend = oracle_mod.local_alignment(q, r)
        assert (sc, ej) == (esc, eend) and ops is None


def test_local_genome_scale(engine, oracle_mod):
    """A contig against the whole PhiX genome (~5.4 k x 5.4 k cells, 85 strips)."""
    from ovlgraph import aligners
    from ovlgraph.reads import read_genome_from_fasta
    genome = read_genome_from_fasta()
    rng = random.Random(11)
    contig, _ = _genome_pair(rng, genome, 4000, len(genome))
    got = aligners.local_alignment(contig, genome, engine=engine)
    exp = oracle_mod.local_alignment(contig, genome)
    assert got == exp
    assert got[3] > 30000


def test_local_limits(engine):
    from ovlgraph import OvlError
    with pytest.raises(OvlError, match="OVL_E_UNSUPPORTED"):
        engine.local_align("A" * 10, "A" * 10, 2 ** 22, -1, -1)
    assert engine.local_align("", "ACGT")[:5] == (0, 0, 0, 0, 0)

"""The banded seed-and-extend knob's oracle (oracle_overlap_banded; not a reference mode).

Pins the C statement against the pure-Python one, and checks the two properties
that tie it to the reference: identical to the full DP (aligners.py:27-57) when
the band covers every diagonal, and identical to the ungapped closed form at
the default indel = -2**31 for ANY band (the seed cell is always in the band).
"""
import random

import numpy as np
import pytest


def _indel_reads(rng, n_reads, max_len, p_sub=0.08, p_indel=0.03):
    base = "".join(rng.choice("ACGT") for _ in range(max_len * 3))
    out = []
    for _ in range(n_reads):
        st = rng.randrange(0, 2 * max_len)
        r = []
        for ch in base[st:st + rng.randint(1, max_len)]:
            u = rng.random()
            if u < p_indel / 2:
                continue                      # deletion
            if u < p_indel:
                r.append(rng.choice("ACGT"))  # insertion
            r.append(rng.choice("ACGT") if rng.random() < p_sub else ch)
        out.append("".join(r) or "A")
    return out


@pytest.fixture(scope="module")
def case():
    rng = random.Random(11)
    reads = _indel_reads(rng, 70, 70) + ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 30)))
                                         for _ in range(10)]
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(400)], np.int32)
    b = np.array([rng.randrange(n) for _ in range(400)], np.int32)
    return reads, a, b


@pytest.mark.parametrize("params", [(10, -1, -2), (1, -1, -1), (3, -2, -5)])
@pytest.mark.parametrize("band", [0, 1, 3, 8, 40])
def test_c_matches_python_statement(oracle_mod, case, params, band):
    reads, a, b = case
    sc, en = oracle_mod.batch_banded(reads, a, b, *params, band)
    for p in range(0, a.shape[0], 5):
        assert (sc[p], en[p]) == oracle_mod.banded_py(reads[a[p]], reads[b[p]], *params, band)


@pytest.mark.parametrize("params", [(10, -1, -2), (1, -1, -1), (2, -3, -1)])
def test_full_band_is_the_reference_dp(oracle_mod, case, params):
    reads, a, b = case
    lmax = max(len(r) for r in reads)
    sc, en = oracle_mod.batch_banded(reads, a, b, *params, 2 * lmax)
    rs, re_ = oracle_mod.batch_dp(reads, a, b, *params)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("band", [0, 2, 17])
def test_default_indel_any_band_is_exact(oracle_mod, case, band):
    reads, a, b = case
    sc, en = oracle_mod.batch_banded(reads, a, b, 10, -1, -(2 ** 31), band)
    rs, re_ = oracle_mod.batch_dp(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_score_monotone_in_band(oracle_mod, case):
    reads, a, b = case
    prev = None
    for band in (0, 1, 2, 4, 8, 16, 200):
        sc, _ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, band)
        if prev is not None:
            assert (sc >= prev).all()
        prev = sc

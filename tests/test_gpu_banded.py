"""GPU banded seed-and-extend knob (band >= 0) vs its oracle, bit-exact.

The band is the build's perf knob for the config-5 sweep, not a
reference mode: parity with the reference holds at full width and at the
default indel; narrower bands are checked against oracle_overlap_banded.
"""
import random

import numpy as np
import pytest

from test_oracle_banded import _indel_reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    from ovlgraph import OverlapEngine
    eng = OverlapEngine(0)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def reads_pairs():
    rng = random.Random(23)
    # lengths up to 250: several 64-row strips, band edges inside and outside the table
    reads = _indel_reads(rng, 300, 250) + _indel_reads(rng, 100, 40)
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(4000)], np.int32)
    b = np.array([rng.randrange(n) for _ in range(4000)], np.int32)
    return reads, a, b


@pytest.mark.parametrize("band", [0, 1, 2, 5, 8, 16, 31, 32, 63, 64, 65, 100, 200])
def test_banded_vs_oracle(engine, oracle_mod, reads_pairs, band):
    reads, a, b = reads_pairs
    engine.set_reads(reads)
    assert engine.plan(10, -1, -2, band) == "banded"
    sc, en = engine.score(a, b, 10, -1, -2, band)
    rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, band)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("params", [(1, -1, -1), (2, -3, -5), (5, -4, -1), (10, -1, -30)])
@pytest.mark.parametrize("band", [3, 24])
def test_banded_params_vs_oracle(engine, oracle_mod, reads_pairs, params, band):
    reads, a, b = reads_pairs
    engine.set_reads(reads)
    sc, en = engine.score(a, b, *params, band)
    rs, re_ = oracle_mod.batch_banded(reads, a, b, *params, band)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_band_at_default_indel_is_exact(engine, oracle_mod, reads_pairs):
    reads, a, b = reads_pairs
    engine.set_reads(reads)
    assert engine.plan(band=4) == engine.plan()
    sc, en = engine.score(a, b, band=4)
    rs, re_ = oracle_mod.batch_dp(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_full_width_band_is_the_reference_dp(engine, oracle_mod, reads_pairs):
    reads, a, b = reads_pairs
    engine.set_reads(reads)
    lmax = max(len(r) for r in reads)
    assert engine.plan(10, -1, -2, 2 * lmax) == "dp"
    sc, en = engine.score(a, b, 10, -1, -2, 2 * lmax)
    rs, re_ = oracle_mod.batch_dp(reads, a, b, 10, -1, -2)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_banded_cfg5_sample(engine, oracle_mod):
    """Config 5 reads (PhiX, l=250, p=0.05): a strided 20k-pair sample at every band of the sweep (4, 8, 16, 32,
    64: one lane per pair up to 32, two lanes per pair at 64), at indel -2 and at the sweep's default indel."""
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg5"))
    a, b = enumerate_candidates(reads, 5)
    idx = np.linspace(0, a.shape[0] - 1, 20000).astype(np.int64)
    a, b = a[idx], b[idx]
    engine.set_reads(reads)
    from ovlgraph.engine import INDEL_DEFAULT
    for indel in (-2, INDEL_DEFAULT):
        for band in (4, 8, 16, 32, 64):
            sc, en = engine.score(a, b, 10, -1, indel, band)
            rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, indel, band)
            np.testing.assert_array_equal(sc, rs, err_msg=f"band {band} indel {indel}")
            np.testing.assert_array_equal(en, re_, err_msg=f"band {band} indel {indel}")


def test_banded_cfg5_full_list(engine, oracle_mod):
    """Config 5 at full size: every one of the 3.38 M candidate pairs at band 8 (the sweep's lane-kernel
    form over the whole list, every tile and length mix), and a 500k strided sample at band 64 (two lanes
    per pair, one row apart: the widest lane-kernel band), against oracle_overlap_banded."""
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg5"))
    a, b = enumerate_candidates(reads, 5)
    engine.set_reads(reads)
    sc, en = engine.score(a, b, 10, -1, -2, 8)
    rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, 8)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)
    idx = np.linspace(0, a.shape[0] - 1, 500_000).astype(np.int64)
    a, b = a[idx], b[idx]
    sc, en = engine.score(a, b, 10, -1, -2, 64)
    rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, 64)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_banded_unsupported_magnitudes(engine):
    from ovlgraph import OvlError
    engine.set_reads(["ACGTACGT", "CGTACGTA"])
    with pytest.raises(OvlError, match="OVL_E_UNSUPPORTED"):
        engine.score([0], [1], 2 ** 28, -1, -1, 4)


FORMS = {"default": {}, "lane": {"OVL_BAND_FORM": "lane"}, "lane1": {"OVL_BAND_FORM": "lane1"},
         "lane2": {"OVL_BAND_FORM": "lane2"}, "diag": {"OVL_BAND_FORM": "diag"},
         "rows": {"OVL_BAND_FORM": "rows"}, "fast": {"OVL_BAND_FORM": "fast"}, "strip": {"OVL_BAND_FORM": "strip"}}


def _score_with_env(env, reads, a, b, params, band):
    import os
    from ovlgraph import OverlapEngine
    os.environ.update(env)
    try:
        with OverlapEngine(0) as eng:
            eng.set_reads(reads)
            return eng.score(a, b, *params, band)
    finally:
        for k in env:
            del os.environ[k]


@pytest.mark.parametrize("band", [0, 1, 2, 3, 8, 15, 16, 31, 32, 33, 63, 64, 95, 96, 150, 255, 256])
@pytest.mark.parametrize("form", sorted(FORMS))
def test_band_forms_agree_with_oracle(oracle_mod, reads_pairs, band, form):
    """The band knob has six kernels: a lane per pair (band <= 32, or <= 64 in steps of 8; the default for
    >= 65,536 pairs), two lanes per pair one row apart (the lane form's choice from band 40; lane1 / lane2
    force either),
    the anti-diagonal form (the default below that), the row form (lanes on band diagonals, a row per
    step; up to 192 lanes), the chunked strip kernel with band masks and the classic strip form,
    picked with OVL_BAND_FORM: each must equal the oracle (lane falls back above band 32)."""
    reads, a, b = reads_pairs
    rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, band)
    sc, en = _score_with_env(FORMS[form], reads, a, b, (10, -1, -2), band)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("band", [5, 40, 100, 300])
def test_banded_long_reads_vs_oracle(engine, oracle_mod, band):
    """Reads past the row form's 1024-base limit, mixed with short ones (seed diagonals far off the
    main one in both directions: bands starting many strips down or many chunks right)."""
    rng = random.Random(31 + band)
    reads = _indel_reads(rng, 40, 1500) + _indel_reads(rng, 40, 90) + _indel_reads(rng, 20, 600)
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(600)], np.int32)
    b = np.array([rng.randrange(n) for _ in range(600)], np.int32)
    engine.set_reads(reads)
    sc, en = engine.score(a, b, 10, -1, -2, band)
    rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, band)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("params", [(10, -1, -2), (1, -1, -1), (2, -3, -5), (5, -4, -1), (10, -1, -30), (3, 2, -1),
                                    (5, -4, 0), (0, 0, -1), (-1, -2, -1), (100, -90, -60), (2, -1, 3)])
@pytest.mark.parametrize("band", [0, 1, 4, 8, 13, 24, 32, 40, 48, 56, 64])
@pytest.mark.parametrize("planes", ["1", "0"])
@pytest.mark.parametrize("lanes", ["1", "2"])
def test_band_lane_kernel_vs_oracle(oracle_mod, params, band, planes, lanes):
    """The band lane kernels over mixed lengths (empty reads, reads shorter than the band, seed
    diagonals left and right of the table) and scorings inside and outside their int8 byte scores
    (those fall back to the anti-diagonal form): one lane per pair (lanes=1) and two lanes per pair one
    row apart (lanes=2; band 0 has one cell and stays on one lane).  planes=1 reads row symbols and t
    codes from the resident bit planes, planes=0 gathers code bytes (OVL_LANE_FORM bit 1)."""
    rng = random.Random(band * 31 + sum(params) % 97)
    lens = [0, 1, 2, 3, 7, 16, 31, 33, 64, 100, 180, 250]
    reads = ["".join(rng.choice("ACGT") for _ in range(rng.choice(lens))) for _ in range(160)]
    reads += _indel_reads(rng, 100, 250)
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(2500)], np.int32)
    b = np.array([rng.randrange(n) for _ in range(2500)], np.int32)
    rs, re_ = oracle_mod.batch_banded(reads, a, b, *params, band)
    sc, en = _score_with_env({"OVL_BAND_FORM": "lane" + lanes, "OVL_LANE_FORM": str(1 + 2 * int(planes))}, reads, a, b, params, band)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)

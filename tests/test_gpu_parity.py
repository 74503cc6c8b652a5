"""GPU parity: the HIP path (through the C ABI) vs the reference's golden vectors and the oracle.

Bit-exact for every comparison (integer scores and end positions).
"""
import contextlib
import io
import random

import numpy as np
import pytest

from conftest import assert_graph_matches_record

pytestmark = pytest.mark.gpu

INDEL = -(2 ** 31)


@pytest.fixture(scope="module")
def engine():
    from ovlgraph import OverlapEngine
    eng = OverlapEngine(0)
    yield eng
    eng.close()


def _pairs_to_reads(pairs):
    reads = []
    for p in pairs:
        reads += [p["s"], p["t"]]
    a = np.arange(0, len(reads), 2, dtype=np.int32)
    return reads, a, a + 1


def _rand(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


# ----------------------------------------------------------------------------- golden vectors

def test_golden_default_batch(engine, golden_default):
    # reads <= 256 bases: bit-plane layout -> ungapped kernel
    pairs = [p for p in golden_default["pairs"] if max(len(p["s"]), len(p["t"])) <= 256]
    assert len(pairs) > 900
    reads, a, b = _pairs_to_reads(pairs)
    engine.set_reads(reads)
    assert engine.plan() == "ungapped"
    sc, en = engine.score(a, b)
    assert sc.tolist() == [p["score"] for p in pairs]
    assert en.tolist() == [p["end"] for p in pairs]
    # every ungapped template tier (wmax 2 / 4 / 8): read sets capped at 64, 128, 256
    for cap in (64, 128):
        sub = [p for p in pairs if max(len(p["s"]), len(p["t"])) <= cap]
        reads, a, b = _pairs_to_reads(sub)
        engine.set_reads(reads)
        assert engine.plan() == "ungapped"
        sc, en = engine.score(a, b)
        assert sc.tolist() == [p["score"] for p in sub]
        assert en.tolist() == [p["end"] for p in sub]


def test_golden_default_through_dp_kernel(engine, golden_default):
    # the gapped kernel must agree in the ungapped regime too (finite but huge indel -> DP plan)
    reads, a, b = _pairs_to_reads(golden_default["pairs"])
    engine.set_reads(reads)
    # indel -2**31 with a 300-base read set forces the DP kernel once lmax > 256
    long_reads = reads + ["A" * 300]
    engine.set_reads(long_reads)
    assert engine.plan() == "dp"
    sc, en = engine.score(a, b)
    assert sc.tolist() == [p["score"] for p in golden_default["pairs"]]
    assert en.tolist() == [p["end"] for p in golden_default["pairs"]]


def test_golden_params(engine, golden_params):
    by_params = {}
    for p in golden_params["pairs"]:
        by_params.setdefault((p["match"], p["mismatch"], p["indel"]), []).append(p)
    for (ma, mm, ind), pairs in by_params.items():
        reads, a, b = _pairs_to_reads(pairs)
        engine.set_reads(reads)
        sc, en = engine.score(a, b, ma, mm, ind)
        assert sc.tolist() == [p["score"] for p in pairs], (ma, mm, ind)
        assert en.tolist() == [p["end"] for p in pairs], (ma, mm, ind)


def test_golden_alphabet(engine, golden_alphabet):
    reads, a, b = _pairs_to_reads(golden_alphabet["pairs"])
    engine.set_reads(reads)
    sc, en = engine.score(a, b)
    assert sc.tolist() == [p["score"] for p in golden_alphabet["pairs"]]
    assert en.tolist() == [p["end"] for p in golden_alphabet["pairs"]]
    # per-alphabet read sets (2-, 4- and 8-plane layouts)
    for lo in range(0, len(golden_alphabet["pairs"]), 30):
        chunk = golden_alphabet["pairs"][lo:lo + 30]
        reads, a, b = _pairs_to_reads(chunk)
        engine.set_reads(reads)
        sc, en = engine.score(a, b)
        assert sc.tolist() == [p["score"] for p in chunk]
        assert en.tolist() == [p["end"] for p in chunk]


def test_overlap_alignment_tuple(engine, golden_default, golden_params, golden_alphabet):
    from ovlgraph.aligners import overlap_alignment
    for p in golden_default["pairs"]:
        if "to_print" in p:
            got = overlap_alignment(p["s"], p["t"], engine=engine)
            assert list(got) == [p["to_print"], p["align_s"], p["align_t"], p["score"], p["end"]]
    for p in golden_params["pairs"][::3]:
        got = overlap_alignment(p["s"], p["t"], p["match"], p["mismatch"], p["indel"], engine=engine)
        assert list(got) == [p["to_print"], p["align_s"], p["align_t"], p["score"], p["end"]]
    for p in golden_alphabet["pairs"][::4]:
        got = overlap_alignment(p["s"], p["t"], engine=engine)
        assert list(got) == [p["to_print"], p["align_s"], p["align_t"], p["score"], p["end"]]


def test_golden_graphs(engine, golden_graphs):
    from ovlgraph import overlapGraphs as og
    for rec in golden_graphs["graphs"]:
        copies = None
        if rec["fn"] == "construct_overlap_graph_nx_k":
            G, copies = og.construct_overlap_graph_nx_k(rec["reads"], engine=engine, **rec["kwargs"])
        elif rec["fn"] == "construct_overlap_graph_string":
            G, copies = og.construct_overlap_graph_string(rec["reads"], engine=engine)
        else:
            with contextlib.redirect_stdout(io.StringIO()):
                G = og.construct_string_graph(rec["reads"], engine=engine)
        assert_graph_matches_record(G, rec, copies)


# ----------------------------------------------------------------------------- seeded vs oracle

@pytest.mark.parametrize("lmax", [1, 5, 20, 31, 32, 33, 64, 65, 96, 100, 128, 129, 150, 160, 192, 200, 224, 255, 256])
def test_random_lengths_vs_oracle(engine, oracle_mod, lmax):
    rng = random.Random(lmax)
    reads = [_rand(rng, rng.randint(1, lmax)) for _ in range(300)]
    reads += [_rand(rng, lmax) for _ in range(100)]
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(4000)], dtype=np.int32)
    b = np.array([rng.randrange(n) for _ in range(4000)], dtype=np.int32)
    engine.set_reads(reads)
    sc, en = engine.score(a, b)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)
    # slice against the full DP restatement too
    ds, de = oracle_mod.batch_dp(reads, a[:400], b[:400])
    np.testing.assert_array_equal(sc[:400], ds)
    np.testing.assert_array_equal(en[:400], de)


def test_overlapping_reads_vs_oracle(engine, oracle_mod):
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    g = read_genome_from_fasta()
    for l, p in ((100, 0.01), (150, 0.02), (250, 0.05), (40, 0.0)):
        reads, _ = dedup_reads(simulate_reads(g, l, 3000, p, seed=l))
        a, b = enumerate_candidates(reads, 5)
        engine.set_reads(reads)
        sc, en = engine.score(a, b)
        rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
        np.testing.assert_array_equal(sc, rs)
        np.testing.assert_array_equal(en, re_)
        assert (sc > 0).mean() > 0.9


@pytest.mark.parametrize("params", [(10, -1, -1), (1, -1, -1), (2, -3, -5), (10, -1, -30), (5, -4, -8)])
def test_gapped_vs_oracle(engine, oracle_mod, params):
    ma, mm, ind = params
    rng = random.Random(sum(params) + 99)
    reads = [_rand(rng, rng.randint(1, 130)) for _ in range(200)]
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(1500)], dtype=np.int32)
    b = np.array([rng.randrange(n) for _ in range(1500)], dtype=np.int32)
    engine.set_reads(reads)
    assert engine.plan(ma, mm, ind) == "dp"
    sc, en = engine.score(a, b, ma, mm, ind)
    rs, re_ = oracle_mod.batch_dp(reads, a, b, ma, mm, ind)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_long_reads_dp_path(engine, oracle_mod):
    rng = random.Random(5)
    reads = [_rand(rng, rng.randint(200, 700)) for _ in range(40)]
    a = np.array([rng.randrange(40) for _ in range(120)], dtype=np.int32)
    b = np.array([rng.randrange(40) for _ in range(120)], dtype=np.int32)
    engine.set_reads(reads)
    assert engine.plan() == "dp"
    sc, en = engine.score(a, b)
    rs, re_ = oracle_mod.batch_dp(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_wide_arithmetic_wraps_like_numba(engine, oracle_mod):
    # magnitudes where int32 stores wrap: the int64 DP kernel must reproduce it
    rng = random.Random(77)
    reads = [_rand(rng, rng.randint(1, 40)) for _ in range(60)]
    a = np.array([rng.randrange(60) for _ in range(300)], dtype=np.int32)
    b = np.array([rng.randrange(60) for _ in range(300)], dtype=np.int32)
    engine.set_reads(reads)
    for ma, mm, ind in ((2 ** 28, -(2 ** 28), -(2 ** 27)), (2 ** 30, -1, -(2 ** 33)), (7, -3, -(2 ** 40))):
        sc, en = engine.score(a, b, ma, mm, ind)
        rs, re_ = oracle_mod.batch_dp(reads, a, b, ma, mm, ind)
        np.testing.assert_array_equal(sc, rs)
        np.testing.assert_array_equal(en, re_)


def test_traceback_matches_oracle(engine, oracle_mod):
    rng = random.Random(3)
    for params in ((10, -1, -1), (10, -1, INDEL), (2, -3, -5)):
        for _ in range(10):
            s, t = _rand(rng, rng.randint(0, 50)), _rand(rng, rng.randint(0, 50))
            engine.set_reads([s, t])
            got = engine.align_one(0, 1, len(s), len(t), *params, traceback=True)
            want = oracle_mod.dp_one(s, t, *params, want_tb=True)
            assert got[:2] == want[:2]
            np.testing.assert_array_equal(got[2], want[2])


# ----------------------------------------------------------------------------- edge cases

def test_empty_and_degenerate(engine):
    engine.set_reads(["", "A", "ACGT", ""])
    sc, en = engine.score([0, 1, 2, 0, 3, 2], [1, 0, 3, 0, 2, 2])
    assert sc.tolist() == [0, 0, 0, 0, 0, 40]
    assert en.tolist() == [0, 0, 0, 0, 0, 4]
    sc, en = engine.score(np.zeros(0, np.int32), np.zeros(0, np.int32))
    assert sc.size == 0


def test_errors(engine):
    from ovlgraph import OvlError
    engine.set_reads(["ACGT", "CGTA"])
    with pytest.raises(OvlError, match="OVL_E_INDEX"):
        engine.score([0, 2], [1, 0])
    with pytest.raises(OvlError, match="OVL_E_UNSUPPORTED"):
        engine.score([0], [1], 2 ** 28, -1, -1, 3)   # banded, scores too large for int32 cells
    with pytest.raises(OvlError, match="OVL_E_ARG"):
        engine.score([0, 1], [1])


def test_device_api_flags_bad_index(engine):
    import torch
    from ovlgraph import OvlError
    engine.set_reads(["ACGTACGT", "CGTACGTA", "TTTT"])
    a = torch.tensor([0, 1, 5, 2], dtype=torch.int32, device="cuda")
    b = torch.tensor([1, 0, 0, -1], dtype=torch.int32, device="cuda")
    s = torch.empty(4, dtype=torch.int32, device="cuda")
    e = torch.empty(4, dtype=torch.int32, device="cuda")
    engine.score_tensors(a, b, s, e)
    with pytest.raises(OvlError, match="OVL_E_INDEX"):
        engine.check_device_errors()
    assert s.cpu().tolist()[2:] == [-1, -1] and e.cpu().tolist()[2:] == [-1, -1]
    engine.check_device_errors()  # flag cleared


def test_one_shot_abi(oracle_mod):
    import ctypes
    from ovlgraph import _lib
    from ovlgraph.engine import encode_reads
    L = _lib.load()
    ctx = ctypes.c_void_p()
    _lib.check(L.ovl_create(0, ctypes.byref(ctx)))
    reads = ["ACGTACGTTT", "GTTTACGA", "TTACG", "CCCC"]
    buf, offs = encode_reads(reads)
    a = np.array([0, 1, 2, 3, 0], np.int32)
    b = np.array([1, 2, 0, 0, 0], np.int32)
    sc = np.zeros(5, np.int32)
    en = np.zeros(5, np.int32)
    p = lambda x: ctypes.c_void_p(x.ctypes.data)
    _lib.check(L.ovl_score_pairs(ctx, p(buf), p(offs), 4, p(a), p(b), 5, 10, -1, INDEL, -1, p(sc), p(en)), ctx)
    rs, re_ = oracle_mod.batch_dp(reads, a, b)
    assert sc.tolist() == rs.tolist() and en.tolist() == re_.tolist()
    L.ovl_destroy(ctx)


# ----------------------------------------------------------------------------- full-size configs

@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "target"])
def test_full_config_vs_oracle(engine, oracle_mod, cfg):
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import CONFIGS, config_reads
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    a, b = enumerate_candidates(reads, CONFIGS[cfg]["k"])
    engine.set_reads(reads)
    sc, en = engine.score(a, b)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)
    # determinism and permutation invariance (size-independent properties)
    perm = np.random.default_rng(1).permutation(a.shape[0])
    sc2, en2 = engine.score(a[perm], b[perm])
    np.testing.assert_array_equal(sc2, sc[perm])
    np.testing.assert_array_equal(en2, en[perm])
    # a slice through the full-DP restatement (the reference recurrence itself)
    ds, de = oracle_mod.batch_dp(reads, a[:2000], b[:2000])
    np.testing.assert_array_equal(sc[:2000], ds)
    np.testing.assert_array_equal(en[:2000], de)


@pytest.mark.parametrize("lw", [1, 7, 31, 32, 33, 63, 64, 95, 96, 97, 100, 127, 128, 150, 160, 192, 224, 250, 256])
@pytest.mark.parametrize("trunc", [0.0, 0.03, 0.5])
def test_uniform_length_sets_vs_oracle(engine, oracle_mod, lw, trunc):
    """Read sets of one dominant length (the uniform kernel) with a fraction of truncated reads
    (the side ring), over every W tier and both sides of the block cut r <= lw - 32(W-1)."""
    rng = random.Random(lw * 1000 + int(trunc * 100))
    reads = [_rand(rng, lw) if rng.random() >= trunc else _rand(rng, rng.randint(1, lw)) for _ in range(700)]
    # related reads so that scores are large and ties frequent
    base = _rand(rng, 3 * lw)
    reads += [base[i:i + lw] for i in range(0, 2 * lw, max(1, lw // 7))]
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(9000)], dtype=np.int32)
    b = np.array([rng.randrange(n) for _ in range(9000)], dtype=np.int32)
    engine.set_reads(reads)
    assert engine.plan() == "ungapped"
    sc, en = engine.score(a, b)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("params", [(1, -1), (3, -2), (127, -1), (10, -120), (2000, -3000)])
def test_uniform_kernel_key_variants(engine, oracle_mod, params):
    """Other match/mismatch values: folded 32-bit keys, and 64-bit keys when scores can reach 2^15."""
    ma, mm = params
    rng = random.Random(ma * 7 + mm)
    reads = [_rand(rng, 100) for _ in range(300)] + [_rand(rng, rng.randint(1, 99)) for _ in range(20)]
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(4000)], dtype=np.int32)
    b = np.array([rng.randrange(n) for _ in range(4000)], dtype=np.int32)
    engine.set_reads(reads)
    indel = -(2 ** 40)
    assert engine.plan(ma, mm, indel) == "ungapped"
    sc, en = engine.score(a, b, ma, mm, indel)
    rs, re_ = oracle_mod.batch_dp(reads, a, b, ma, mm, indel)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("n_short", [1, 12, 60])
def test_clustered_side_pairs_vs_oracle(engine, oracle_mod, n_short):
    """Candidate lists in read order, as overlapGraphs.py:43-53 emits them: the pairs of a truncated
    read are consecutive, so whole tiles of side pairs reach one latency-mode side wave (drained at
    raised issue priority) or one throughput-mode ring."""
    rng = random.Random(7 + n_short)
    reads = [_rand(rng, 100) for _ in range(300)] + [_rand(rng, rng.randint(1, 99)) for _ in range(n_short)]
    rng.shuffle(reads)
    n = len(reads)
    a, b = [], []
    for i in range(n):
        for j in rng.sample(range(n), 40):
            if j != i:
                a.append(i)
                b.append(j)
    a = np.array(a, dtype=np.int32)
    b = np.array(b, dtype=np.int32)
    engine.set_reads(reads)
    assert engine.plan() == "ungapped"
    sc, en = engine.score(a, b)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("n_pairs", [100_000, 400_000])
def test_latency_and_throughput_modes(oracle_mod, n_pairs):
    """The planner's two uniform-kernel modes give the reference's results: latency mode (a side-pair
    wavefront beside each sweeping one) up to 8 tiles per CU (131,072 pairs on 256 CUs), throughput mode
    above -- 400,000 pairs (6,250 tiles) also make its blocks loop over tiles."""
    from ovlgraph import OverlapEngine
    rng = random.Random(42)
    reads = [_rand(rng, 100) for _ in range(400)] + [_rand(rng, rng.randint(1, 99)) for _ in range(30)]
    n = len(reads)
    nr = np.random.default_rng(42)
    a = nr.integers(0, n, n_pairs, dtype=np.int32)
    b = nr.integers(0, n, n_pairs, dtype=np.int32)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        sc, en = eng.score(a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("lw", [31, 32, 64, 100, 128, 150, 250])
@pytest.mark.parametrize("split", ["0", "1"])
def test_t_truncated_pairs_in_sweep(oracle_mod, lw, split):
    """Pairs (full-length a, truncated b) are scored inside the uniform sweep (snapshot of block m/32
    after shift m % 32): every m in 0..lw-1, b cut from a's continuation so that the best end sits at
    or next to m, in throughput mode ("0": 200,000 pairs, above 8 tiles per CU) and latency mode ("1":
    120,000 pairs), several truncated lanes per wavefront with equal and distinct m % 32."""
    from ovlgraph import OverlapEngine
    rng = random.Random(lw * 3 + int(split))
    n_list = 200_000 if split == "0" else 120_000
    genome = _rand(rng, 40 * lw)
    starts = list(range(0, 30 * lw, max(1, lw // 5)))
    full = [genome[i:i + lw] for i in starts]
    short = []
    for m in range(1, lw):
        st = rng.choice(starts)
        short.append(genome[st:st + m])                     # prefix of a full read: overlaps end at or near m
        short.append(_rand(rng, m))                          # unrelated
    reads = full + short
    n_full, n = len(full), len(reads)
    nr = np.random.default_rng(lw)
    a = nr.integers(0, n_full, n_list, dtype=np.int32)
    b = np.where(nr.random(n_list) < 0.3, nr.integers(n_full, n, n_list), nr.integers(0, n, n_list)).astype(np.int32)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        assert eng.plan() == "ungapped"
        sc, en = eng.score(a, b)
        sc_small, en_small = eng.score(a[:3000], b[:3000])
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)
    np.testing.assert_array_equal(sc_small, rs[:3000])
    np.testing.assert_array_equal(en_small, re_[:3000])


@pytest.mark.parametrize("params", [(10, -1, -2), (1, -1, -1), (2, -3, -5), (2 ** 28, -(2 ** 28), -(2 ** 27))])
def test_dp_fast_and_classic_agree_with_oracle(oracle_mod, params):
    """Scores-only full DP runs dp_fast_kernel (chunked, unrolled); OVL_DP_FORM=classic forces dp_kernel.
    Lengths cross 64-row strips and 64-column chunks on both axes; the last set wraps int32 stores."""
    import os
    from ovlgraph import OverlapEngine
    rng = random.Random(sum(abs(x) for x in params) % 1000 + 5)
    lens = [1, 2, 62, 63, 64, 65, 127, 128, 129, 191, 200, 257, 300]
    reads = [_rand(rng, rng.choice(lens)) for _ in range(120)] + [_rand(rng, rng.randint(1, 320)) for _ in range(80)]
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(900)], dtype=np.int32)
    b = np.array([rng.randrange(n) for _ in range(900)], dtype=np.int32)
    rs, re_ = oracle_mod.batch_dp(reads, a, b, *params)
    for form in ("fast", "classic"):
        os.environ["OVL_DP_FORM"] = form
        try:
            with OverlapEngine(0) as eng:
                eng.set_reads(reads)
                assert eng.plan(*params) == "dp"
                sc, en = eng.score(a, b, *params)
        finally:
            del os.environ["OVL_DP_FORM"]
        np.testing.assert_array_equal(sc, rs)
        np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("case", ["acgt_odd_total", "subset_AT", "subset_CG_T", "n_at_end", "n_at_start",
                                  "lowercase", "tiny"])
def test_read_upload_forms(engine, oracle_mod, case):
    """ovl_set_reads uploads ACGT-only read sets 2-bit packed (stage_reads, unpack2_kernel) and any other
    byte set as it is: odd totals (not a multiple of 4 or 64 bytes), alphabets that are strict subsets of ACGT
    (their dense codes differ from A C G T = 0 1 2 3), a single other byte at either end of the bytes (the
    packing abandoned in the last or the first part), lowercase, a few bases -- all equal to the oracle."""
    rng = random.Random(sum(map(ord, case)))
    alpha = {"subset_AT": "AT", "subset_CG_T": "CGT", "lowercase": "acgt"}.get(case, "ACGT")
    n = 3 if case == "tiny" else 3001
    reads = [_rand(rng, rng.randint(1, 7) if case == "tiny" else rng.choice([97, 100, 101, 100, 33]), alpha)
             for _ in range(n)]
    if case == "n_at_end":
        reads[-1] = reads[-1][:-1] + "N"
    if case == "n_at_start":
        reads[0] = "N" + reads[0][1:]
    m = 40_000 if n > 3 else 9
    a = np.array([rng.randrange(n) for _ in range(m)], np.int32)
    b = np.array([rng.randrange(n) for _ in range(m)], np.int32)
    engine.set_reads(reads)
    s, e = engine.score(a, b)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b, 10, -1)
    np.testing.assert_array_equal(s, rs)
    np.testing.assert_array_equal(e, re_)
    # the gapped kernels read the same codes
    s2, e2 = engine.score(a[:2000], b[:2000], indel=-2)
    rs2, re2 = oracle_mod.batch_dp(reads, a[:2000], b[:2000], 10, -1, -2)
    np.testing.assert_array_equal(s2, rs2)
    np.testing.assert_array_equal(e2, re2)

"""GPU: host pair lists in compact form (ovl_pairs.hip, ovl_api.cpp encode_chunk).

ovl_score_host / ovl_score_pairs encode the caller's int32 pairs per pipeline chunk -- b as uint16 when
n_reads <= 65,535; a, when the list is a-major (overlapGraphs.py:43-52), as tile deltas that uniform_kernel
reads in place (IX: a = base[p / 64] + d8[p]) or as runs that kernels decode into HBM.  Every result is
compared with the oracle and with the uncompressed path (OVL_PAIRS_FORM=plain): a-major and shuffled lists
(in place / runs / no runs), uint16 and int32 widths, pinned and pageable lists, odd chunk sizes, tiles whose
a jumps past the delta range, calls small enough for the latency-mode launch, and bad indices (OVL_E_INDEX,
-1 results, the rest exact).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine_env(env):
    from ovlgraph import OverlapEngine
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return OverlapEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def target():
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("target", seed=0))
    a, b = enumerate_candidates(reads, 5)
    return reads, a, b


@pytest.mark.parametrize("order", ["reference", "shuffled"])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("chunk", [None, "300007"])
def test_compact_vs_oracle_and_plain(oracle_mod, target, order, pinned, chunk):
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = target
    if order == "shuffled":
        perm = np.random.default_rng(1).permutation(a.shape[0])
        a, b = a[perm], b[perm]
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
    if pinned:
        pa, pb = pinned_empty(a.shape[0]), pinned_empty(b.shape[0])
        pa[:], pb[:] = a, b
        a, b = pa, pb
    env = {"OVL_PIPE_CHUNK": chunk} if chunk else {}
    comp = _engine_env(env)
    plain = _engine_env(dict(env, OVL_PAIRS_FORM="plain"))
    try:
        for e in (comp, plain):
            e.set_reads(reads)
        for _ in range(2):
            s, en = comp.score(a, b)
            np.testing.assert_array_equal(s, ref_s)
            np.testing.assert_array_equal(en, ref_e)
        x = comp.last_transfer()
        s2, e2 = plain.score(a, b)
        np.testing.assert_array_equal(s2, ref_s)
        np.testing.assert_array_equal(e2, ref_e)
        y = plain.last_transfer()
        # the compact list moves fewer bytes over the link (b in 16 bits, a-major lists as runs)
        assert x["link_bytes"] < y["link_bytes"], (x, y)
    finally:
        comp.close()
        plain.close()


def test_compact_int32_width_cfg4_sample(oracle_mod):
    """More than 65,535 reads: b (and a when not in runs) cross as int32; the a-major runs still apply."""
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg4", seed=0))
    assert len(reads) > 65535
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        a, b = eng.candidates(5)
        a, b = np.array(a[:3_000_000]), np.array(b[:3_000_000])
        s, e = eng.score(a, b)
        idx = np.linspace(0, a.shape[0] - 1, 200_000).astype(np.int64)
        rs, re_ = oracle_mod.batch_closed_form(reads, a[idx], b[idx])
        np.testing.assert_array_equal(s[idx], rs)
        np.testing.assert_array_equal(e[idx], re_)
        cs, ce = eng.score_candidates_range(0, 3_000_000)
        np.testing.assert_array_equal(s, cs)
        np.testing.assert_array_equal(e, ce)


@pytest.mark.parametrize("bad", [-1, "n", 70000, -(2 ** 31), 2 ** 31 - 1])
def test_compact_bad_indices(oracle_mod, target, bad):
    from ovlgraph import OverlapEngine, OvlError
    reads, a, b = target
    n = len(reads)
    v = n if bad == "n" else bad
    a, b = a.copy(), b.copy()
    hit_a = np.array([0, 5, 123_457, a.shape[0] - 1])
    hit_b = np.array([77, 400_001, 1_500_000])
    a[hit_a] = v
    b[hit_b] = v
    bad_mask = np.zeros(a.shape[0], bool)
    bad_mask[hit_a] = True
    bad_mask[hit_b] = True
    ok = ~bad_mask
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a[ok], b[ok])
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        out = (np.full(a.shape[0], 7, np.int32), np.full(a.shape[0], 7, np.int32))
        with pytest.raises(OvlError, match="OVL_E_INDEX"):
            eng.score(a, b, out=out)
        np.testing.assert_array_equal(out[0][bad_mask], -1)
        np.testing.assert_array_equal(out[1][bad_mask], -1)
        np.testing.assert_array_equal(out[0][ok], ref_s)
        np.testing.assert_array_equal(out[1][ok], ref_e)
        # the context recovers: a clean call right after
        s, e = eng.score(a[ok][:100_000], b[ok][:100_000])
        np.testing.assert_array_equal(s, ref_s[:100_000])


def test_one_shot_abi_call(oracle_mod, target):
    """ovl_score_pairs (reads + pair list in host memory) through the compact path, twice (stage reuse),
    then a smaller read set on the same context."""
    from ovlgraph import OverlapEngine
    reads, a, b = target
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
    with OverlapEngine(0) as eng:
        for _ in range(2):
            s, e = eng.score_pairs(reads, a, b)
            np.testing.assert_array_equal(s, ref_s)
            np.testing.assert_array_equal(e, ref_e)
        small = reads[:3000]
        keep = (a < 3000) & (b < 3000)
        s, e = eng.score_pairs(small, a[keep], b[keep])
        rs, re_ = oracle_mod.batch_closed_form(small, a[keep], b[keep])
        np.testing.assert_array_equal(s, rs)
        np.testing.assert_array_equal(e, re_)


@pytest.mark.parametrize("pack", ["1", "0"])
def test_compact_adaptive_share(oracle_mod, target, pack):
    """Host-list calls into pinned arrays: 2-byte packing (OVL_PACK=1, the default) keeps its own adaptive direct
    share (the host also encodes the list), the packed part within 20-98 % of the pairs; OVL_PACK=0 packs none.
    Exact results call after call."""
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = target
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
    n = a.shape[0]
    with _engine_env({"OVL_PACK": pack}) as eng:
        eng.set_reads(reads)
        out = (pinned_empty(n), pinned_empty(n))
        shares = []
        for _ in range(12):
            out[0][:] = -9
            eng.score(a, b, out=out)
            np.testing.assert_array_equal(out[0], ref_s)
            np.testing.assert_array_equal(out[1], ref_e)
            shares.append(eng.last_transfer()["packed_pairs"] / n)
        if pack == "1":
            assert all(0.19 <= x <= 0.99 for x in shares), shares
        else:
            assert all(x == 0.0 for x in shares), shares


def _pair_link_bytes(eng, n):
    """Bytes of the pair list that crossed the link in the last call (the results' bytes subtracted,
    ovl_last_results)."""
    t = eng.last_transfer()
    return t["link_bytes"] - t["result_bytes"]


@pytest.mark.parametrize("pinned", [False, True])
def test_ix_in_place_vs_decode(oracle_mod, target, pinned):
    """The a-major target list is read in place (3 B per pair + 4 B per tile); OVL_PAIRS_FORM=decode decodes the
    same encoding's runs into HBM first.  Same results; the path each call took is asserted from
    ovl_last_pair_list (pairs read in place / decoded), not inferred from its link bytes."""
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = target
    n = a.shape[0]
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
    if pinned:
        pa, pb = pinned_empty(n), pinned_empty(n)
        pa[:], pb[:] = a, b
        a, b = pa, pb
    ix = _engine_env({})
    dec = _engine_env({"OVL_PAIRS_FORM": "decode"})
    try:
        for e in (ix, dec):
            e.set_reads(reads)
        for _ in range(3):
            s, en = ix.score(a, b)
            np.testing.assert_array_equal(s, ref_s)
            np.testing.assert_array_equal(en, ref_e)
            got = ix.last_pair_list()
            assert got == {"in_place_pairs": n, "decoded_pairs": 0}, (got, ix.plan(), ix.info(), ix.last_transfer(),
                                                                      {k: v for k, v in os.environ.items()
                                                                       if k.startswith("OVL")})
        s, en = dec.score(a, b)
        np.testing.assert_array_equal(s, ref_s)
        np.testing.assert_array_equal(en, ref_e)
        assert dec.last_pair_list() == {"in_place_pairs": 0, "decoded_pairs": n}
        assert _pair_link_bytes(dec, n) < 3 * n  # b16 + runs
    finally:
        ix.close()
        dec.close()


def test_ix_tile_jumps_fall_back(oracle_mod, target):
    """An a-major list whose a jumps by more than 255 inside some tiles: those chunks take the runs decode,
    the others stay in place; exact either way."""
    reads, _, _ = target
    nr = len(reads)
    rng = np.random.default_rng(5)
    n = 1_200_000
    # a non-decreasing over [0, nr) with runs of ~40, plus a few jumps of 300-2000 inside tiles
    steps = (rng.random(n) < 1 / 40).astype(np.int64)
    jump_at = rng.choice(n, 6, replace=False)
    steps[jump_at] = rng.integers(300, 2000, 6)
    a = np.cumsum(steps)
    a = (a * (nr - 1) // max(int(a[-1]), 1)).astype(np.int32)
    b = rng.integers(0, nr, n, dtype=np.int32)
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
    eng = _engine_env({})
    try:
        eng.set_reads(reads)
        s, e = eng.score(a, b)
        np.testing.assert_array_equal(s, ref_s)
        np.testing.assert_array_equal(e, ref_e)
        got = eng.last_pair_list()
        assert got["decoded_pairs"] > 0 and sum(got.values()) == n, got  # the chunks with a jump took the runs
    finally:
        eng.close()


@pytest.mark.parametrize("pack", ["1", "0"])
def test_ix_small_call_latency_mode(oracle_mod, target, pack):
    """100 K pairs, compact: few enough for the latency-mode launch, which takes the decoded list (runs: < 3 B per
    pair), with 2-byte packed results (OVL_PACK=1) and with int32 results (OVL_PACK=0)."""
    reads, a, b = target
    a, b = a[:100_000], b[:100_000]
    n = a.shape[0]
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
    eng = _engine_env({"OVL_PACK": pack})
    try:
        eng.set_reads(reads)
        s, e = eng.score(a, b)
        np.testing.assert_array_equal(s, ref_s)
        np.testing.assert_array_equal(e, ref_e)
        assert _pair_link_bytes(eng, n) < 3 * n
        assert eng.last_pair_list() == {"in_place_pairs": 0, "decoded_pairs": n}
    finally:
        eng.close()


def test_ix_cfg3_width5(oracle_mod):
    """cfg3 (l = 150, W = 5 words per row) through the in-place list: equal to the resident-list scoring and
    to the oracle on a sample."""
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg3", seed=0))
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        a, b = eng.candidates(5)
        a, b = np.array(a), np.array(b)
        n = a.shape[0]
        s, e = eng.score(a, b)
        lb = _pair_link_bytes(eng, n)
        assert 3 * n + 4 * (n // 64) <= lb <= 3 * n + 4 * (n // 64 + 64), lb
        cs, ce = eng.score_candidates()
        np.testing.assert_array_equal(s, cs)
        np.testing.assert_array_equal(e, ce)
        idx = np.linspace(0, n - 1, 150_000).astype(np.int64)
        rs, re_ = oracle_mod.batch_closed_form(reads, a[idx], b[idx])
        np.testing.assert_array_equal(s[idx], rs)
        np.testing.assert_array_equal(e[idx], re_)

"""GPU parity of the lane-per-pair full DP (csrc/ovl_dp_lane.hip) for gapped scoring.

aligners.py:27-57 with a finite indel: every (score, end) must equal the oracle's C
restatement bit for bit.  OVL_DP_FORM=lane forces the lane kernel for small lists (the
planner picks it automatically only for >= 65,536 pairs).
Wavefronts mix read lengths (virtual leading rows), lengths cross the 32-column strips,
and the list length is not a multiple of 64.
"""
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rand(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


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


LENS = [0, 1, 2, 3, 4, 5, 15, 16, 17, 31, 32, 33, 47, 63, 64, 65, 100, 127, 128, 129, 250, 251, 255]


@pytest.fixture(scope="module", params=[256, 260])
def mixed_set(request):
    """lmax 256: bit-plane layouts exist (row symbols from the planes, the LDS hand-off); 260: they do not."""
    lmax = request.param
    rng = random.Random(2024 + lmax)
    reads = [_rand(rng, rng.choice(LENS)) for _ in range(150)] + [_rand(rng, rng.randint(1, lmax)) for _ in range(150)]
    reads[0] = _rand(rng, lmax)
    n = len(reads)
    a = np.array([rng.randrange(n) for _ in range(3001)], dtype=np.int32)
    b = np.array([rng.randrange(n) for _ in range(3001)], dtype=np.int32)
    return reads, a, b


# byte score profile x bit-plane row symbols; the hand-off column form follows the scoring (4-bit steps in LDS
# when the profile and planes are on, the steps are bounded by 15 and lmax <= 256; else int16 or int32 in HBM),
# so the 13 scorings below reach every form
VARIANTS = {f"prof{pr}-sfx{sx}": {"OVL_LANE_FORM": str(int(pr) + 2 * int(sx))}
            for pr in ("0", "1") for sx in ("0", "1") if pr == "1" or sx == "0"}
# the default form: with the LDS hand-off, two pairs per lane as packed f16 cells (dp_lane_h2_kernel) when both
# diagonal scores' f16 encodings end in a zero byte -- (10, -1, -2), (1, -1, -1), (3, 2, -1), (-1, -2, -1),
# (2, -1, 0), (2, -3, -5), (8, -8, -3) and (12, -4, -1) below
VARIANTS["prof1-sfx1-h2"] = {"OVL_LANE_FORM": "7"}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("params", [(10, -1, -2), (1, -1, -1), (2, -3, -5), (10, -1, -30), (5, -4, -8), (3, 2, -1),
                                    (-1, -2, -1), (0, 0, -1), (100, -90, -60), (1000, -1, -3), (2, -1, 0),
                                    (2, -1, 1), (-3, -5, 2), (8, -8, -3), (12, -4, -1)])
def test_lane_vs_oracle_mixed_lengths(oracle_mod, mixed_set, params, variant):
    """(100, -90, -60) and (1000, -1, -3) leave the int8 profile and the int16 column, and a positive
    indel leaves the zero-profile virtual rows: those fall back to compare/select, masked virtual rows
    and int32 inside the same kernel family."""
    reads, a, b = mixed_set
    rs, re_ = oracle_mod.batch_dp(reads, a, b, *params)
    with _engine_env(dict(VARIANTS[variant], OVL_DP_FORM="lane")) as eng:
        eng.set_reads(reads)
        # (0, 0, -1) over bit-plane reads is the closed form (gaps cannot win): still checked
        assert eng.plan(*params) == "dp" or params == (0, 0, -1)
        sc, en = eng.score(a, b, *params)
        eng.check_device_errors()
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_lane_uniform_reads_with_truncated_tail(oracle_mod, variant):
    """The benchmark shape: reads of one length, a few truncated (genome end), overlapping."""
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    reads, _ = dedup_reads(simulate_reads(read_genome_from_fasta(), 250, 600, 0.05, seed=3))
    a, b = enumerate_candidates(reads, 5)
    a, b = a[:4000], b[:4000]
    rs, re_ = oracle_mod.batch_dp(reads, a, b, 10, -1, -2)
    with _engine_env(dict(VARIANTS[variant], OVL_DP_FORM="lane")) as eng:
        eng.set_reads(reads)
        sc, en = eng.score(a, b, 10, -1, -2)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


@pytest.mark.parametrize("params", [(10, -1, -2), (12, -4, -1), (8, -8, -3)])
def test_lane_h2_vs_int32_at_scale(oracle_mod, params):
    """BASELINE configs[4]'s shape (l = 250, p = 0.05), >= 65,536 pairs: the packed-f16 two-pairs-per-lane
    kernel (default) equals the int32 lane kernel (OVL_LANE_FORM=3) on every pair, and the oracle on a
    strided sample -- long strips through the 32-row offset moves at the largest steps the form takes."""
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    reads, _ = dedup_reads(simulate_reads(read_genome_from_fasta(), 250, 8000, 0.05, seed=11))
    a, b = enumerate_candidates(reads, 5)
    assert a.shape[0] >= 65536
    with _engine_env({}) as eng:
        eng.set_reads(reads)
        sc, en = eng.score(a, b, *params)
    with _engine_env({"OVL_LANE_FORM": "3"}) as eng:
        eng.set_reads(reads)
        s3, e3 = eng.score(a, b, *params)
    np.testing.assert_array_equal(sc, s3)
    np.testing.assert_array_equal(en, e3)
    idx = np.arange(0, a.shape[0], 97)
    rs, re_ = oracle_mod.batch_dp(reads, a[idx], b[idx], *params)
    np.testing.assert_array_equal(sc[idx], rs)
    np.testing.assert_array_equal(en[idx], re_)


def test_lane_wide_alphabet_vs_oracle(oracle_mod):
    """More than 4 symbols (N, lowercase): no byte profile, compare/select on the codes."""
    rng = random.Random(8)
    reads = [_rand(rng, rng.choice(LENS), "ACGTNacgtRY") for _ in range(200)]
    a = np.array([rng.randrange(200) for _ in range(1300)], dtype=np.int32)
    b = np.array([rng.randrange(200) for _ in range(1300)], dtype=np.int32)
    rs, re_ = oracle_mod.batch_dp(reads, a, b, 10, -1, -2)
    with _engine_env({"OVL_DP_FORM": "lane"}) as eng:
        eng.set_reads(reads)
        sc, en = eng.score(a, b, 10, -1, -2)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_lane_and_fast_kernels_agree_at_scale(oracle_mod):
    """>= 65,536 pairs: the planner's automatic choice (lane kernel) equals dp_fast_kernel
    (OVL_DP_FORM=fast) on every pair, and the oracle on a strided sample."""
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import read_genome_from_fasta, simulate_reads
    reads, _ = dedup_reads(simulate_reads(read_genome_from_fasta(), 150, 8000, 0.02, seed=1))
    a, b = enumerate_candidates(reads, 5)
    assert a.shape[0] >= 65536
    with _engine_env({}) as eng:
        eng.set_reads(reads)
        sc, en = eng.score(a, b, 10, -1, -2)
    with _engine_env({"OVL_DP_FORM": "fast"}) as eng:
        eng.set_reads(reads)
        fs, fe = eng.score(a, b, 10, -1, -2)
    np.testing.assert_array_equal(sc, fs)
    np.testing.assert_array_equal(en, fe)
    idx = np.arange(0, a.shape[0], 37)
    rs, re_ = oracle_mod.batch_dp(reads, a[idx], b[idx], 10, -1, -2)
    np.testing.assert_array_equal(sc[idx], rs)
    np.testing.assert_array_equal(en[idx], re_)


def test_lane_falls_back_on_large_magnitudes(oracle_mod, mixed_set):
    """Magnitudes outside the lane kernel's int32 potential bound take the anti-diagonal kernels."""
    reads, a, b = mixed_set
    params = (2 ** 20, -(2 ** 20), -(2 ** 19))
    rs, re_ = oracle_mod.batch_dp(reads, a[:500], b[:500], *params)
    with _engine_env({"OVL_DP_FORM": "lane"}) as eng:
        eng.set_reads(reads)
        sc, en = eng.score(a[:500], b[:500], *params)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)


def test_lane_flags_bad_index(mixed_set):
    import torch
    reads, a, b = mixed_set
    with _engine_env({"OVL_DP_FORM": "lane"}) as eng:
        eng.set_reads(reads)
        da = torch.as_tensor(np.array([0, 1, len(reads) + 5, 2], dtype=np.int32), device="cuda")
        db = torch.as_tensor(np.array([1, 2, 3, -1], dtype=np.int32), device="cuda")
        ds = torch.empty(4, dtype=torch.int32, device="cuda")
        de = torch.empty(4, dtype=torch.int32, device="cuda")
        launch = eng.launcher(da, db, ds, de, 10, -1, -2, -1)
        launch()
        torch.cuda.synchronize()
        assert ds[2].item() == -1 and de[3].item() == -1
        with pytest.raises(Exception):
            eng.check_device_errors()


def test_h2_full_dp_across_launch_slices(oracle_mod):
    """The packed-f16 full DP (dp_lane_h2_kernel) launches at most 2^23 pairs at a time over one reused hand-off
    column buffer (ovl_api.cpp launch_score_chunk, kH2Slice): a device list of 2^24 + 4,099 pairs (cfg2's list
    repeated) scores in three slices with each slice's results where they belong -- checked against the oracle on a
    strided sample and on every pair around the slice boundaries -- and the device memory the call leaves allocated
    stays near one slice's column buffer (64 B per pair at 100-base reads: 0.54 GB), not the list's (1.07 GB)."""
    import torch
    from ovlgraph import OverlapEngine
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg2", seed=0))
    a0, b0 = enumerate_candidates(reads, 5)
    n = (1 << 24) + 4099
    reps = -(-n // a0.shape[0])
    a = np.tile(a0, reps)[:n].astype(np.int32)
    b = np.tile(b0, reps)[:n].astype(np.int32)
    dev = torch.device("cuda", 0)
    with OverlapEngine(0) as eng:
        eng.set_reads(reads)
        assert eng.plan(10, -1, -2) == "dp"
        ta, tb = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        so = torch.empty(n, dtype=torch.int32, device=dev)
        eo = torch.empty(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)
        free0 = torch.cuda.mem_get_info(dev)[0]
        eng.score_tensors(ta, tb, so, eo, 10, -1, -2)
        torch.cuda.synchronize(dev)
        eng.check_device_errors()
        grown = free0 - torch.cuda.mem_get_info(dev)[0]
        assert grown < 0.8e9, grown  # (one slice's buffer and some slack, not the whole list's)
        s, e = so.cpu().numpy(), eo.cpu().numpy()
    idx = np.unique(np.concatenate([np.linspace(0, n - 1, 40_000).astype(np.int64),
                                    np.arange((1 << 23) - 2000, (1 << 23) + 2000),
                                    np.arange((1 << 24) - 2000, n)]))
    rs, re_ = oracle_mod.batch_dp(reads, a[idx], b[idx], 10, -1, -2)
    np.testing.assert_array_equal(s[idx], rs)
    np.testing.assert_array_equal(e[idx], re_)

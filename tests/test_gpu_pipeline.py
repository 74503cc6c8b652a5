"""GPU: the host-array pipeline, multi-device contexts, sharding and gathers, full-size cfg5.

Every result is compared bit for bit with the oracle (oracle/ovl_oracle.c, the restatement of
aligners.py:27-57) or with another path already checked against it.

* ovl_score_host / ovl_score_candidates: chunked H2D / kernel / D2H pipeline, pinned and pageable
  caller arrays, many chunks (staging-slot reuse), device-side index errors.
* ovl_create(0) / ovl_create_on_devices: one context over the visible GPUs (one on this box),
  Σ n·m shard bounds on the device (ovl_candidates_shards) == ovlgraph.sharded.shard_bounds,
  ovl_score_candidates_range shards reassemble the whole list.
* ovlgraph.sharded at world 1 on backend "nccl" (RCCL): score_pairs_sharded, ShardedStep with
  dest="host" (shared pinned host buffer) and dest="rank0" (dist.gather).
* dp_lane_kernel launches on two streams share the hand-off buffer safely.
* cfg5 (BASELINE configs[4], 3.39 M pairs, l = 250) at full size: default scoring vs the oracle's
  closed form; gapped (indel -2) lane kernel == wavefront kernel on the whole list, and both ==
  the oracle's full DP on a 50k-pair strided sample.
"""
import ctypes
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine_env(env, **kw):
    from ovlgraph import OverlapEngine
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return OverlapEngine(**kw) if kw else OverlapEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def cfg2():
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg2", seed=0))
    a, b = enumerate_candidates(reads, 5)
    return reads, a, b


@pytest.fixture(scope="module")
def cfg2_ref(oracle_mod, cfg2):
    reads, a, b = cfg2
    return oracle_mod.batch_ungapped(reads, a, b)


@pytest.fixture(scope="module")
def engine():
    from ovlgraph import OverlapEngine
    eng = OverlapEngine(0)
    yield eng
    eng.close()


@pytest.mark.parametrize("chunk", ["0", "64", "1000", "65536"])
def test_pipeline_host_list_pinned_and_pageable(oracle_mod, cfg2, cfg2_ref, chunk):
    from ovlgraph.hostmem import is_pinned_array, pinned_empty
    reads, a, b = cfg2
    eng = _engine_env({"OVL_PIPE_CHUNK": chunk})
    try:
        eng.set_reads(reads)
        # pageable inputs, pinned outputs (the default)
        sc, en = eng.score(a, b)
        assert is_pinned_array(sc) and is_pinned_array(en)
        np.testing.assert_array_equal(sc, cfg2_ref[0])
        np.testing.assert_array_equal(en, cfg2_ref[1])
        # pageable outputs (staging ring)
        out = (np.full(a.shape[0], 7, np.int32), np.full(a.shape[0], 7, np.int32))
        eng.score(a, b, out=out)
        np.testing.assert_array_equal(out[0], cfg2_ref[0])
        np.testing.assert_array_equal(out[1], cfg2_ref[1])
        # pinned inputs too
        pa, pb = pinned_empty(a.shape[0]), pinned_empty(a.shape[0])
        pa[:] = a
        pb[:] = b
        sc2, en2 = eng.score(pa, pb)
        np.testing.assert_array_equal(sc2, cfg2_ref[0])
        np.testing.assert_array_equal(en2, cfg2_ref[1])
        # resident device list -> pinned and pageable outputs
        da, db = eng.candidates(5)
        np.testing.assert_array_equal(da, a)
        np.testing.assert_array_equal(db, b)
        cs, ce = eng.score_candidates()
        np.testing.assert_array_equal(cs, cfg2_ref[0])
        np.testing.assert_array_equal(ce, cfg2_ref[1])
        out = (np.zeros(a.shape[0] + 5, np.int32), np.zeros(a.shape[0] + 5, np.int32))
        eng.score_candidates(out=out)
        np.testing.assert_array_equal(out[0][: a.shape[0]], cfg2_ref[0])
        assert out[0][a.shape[0]:].tolist() == [0] * 5  # nothing past n_pairs is written
    finally:
        eng.close()


@pytest.mark.parametrize("pack,pct", [("1", "25"), ("1", "0"), ("1", "60"), ("1", "100"), ("0", "25")])
@pytest.mark.parametrize("chunk", ["0", "1000"])
def test_packed_results_host_arrays(oracle_mod, cfg2, cfg2_ref, pack, pct, chunk):
    """Results cross the link packed (uint16 score | end << 8) and are expanded on the host: pinned,
    pageable and misaligned caller arrays, list lengths that are not a multiple of the 8-pair step, staging
    slot reuse (many chunks, 1000-pair chunks that are not a multiple of the 64-pair rounding), bad pairs
    expanded to (-1, -1); pinned arrays with 0-100 % of the pairs in
    direct int32 chunks after the packed ones; OVL_PACK=0 is the int32 transport.  (OVL_PACK_MIN=0: packed
    below the default 1 M-pair threshold; OVL_PAIRS_FORM=plain: the pair list crosses as int32, 8 B/pair --
    the compact encoding has its own tests, test_gpu_compact_pairs.py.)"""
    from ovlgraph import OvlError
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = cfg2
    eng = _engine_env({"OVL_PACK": pack, "OVL_PACK_MIN": "0", "OVL_PACK_DIRECT_PCT": pct,
                       "OVL_PIPE_CHUNK": chunk, "OVL_PAIRS_FORM": "plain"})
    try:
        eng.set_reads(reads)
        n = a.shape[0] - 3
        outs = {"pinned": (pinned_empty(n), pinned_empty(n)),
                "pageable": (np.empty(n, np.int32), np.empty(n, np.int32)),
                # 4-byte offsets: the expansion's 16-byte alignment differs between the two arrays
                "misaligned": (np.empty(n + 1, np.int32)[1:], np.empty(n + 2, np.int32)[2:])}
        for name, out in outs.items():
            out[0][:] = 7
            out[1][:] = 7
            eng.score(a[:n], b[:n], out=out)
            np.testing.assert_array_equal(out[0], cfg2_ref[0][:n], err_msg=name)
            np.testing.assert_array_equal(out[1], cfg2_ref[1][:n], err_msg=name)
            # ovl_last_transfer: the pair list (8 B/pair) plus 2 B per packed and 8 B per other pair
            x = eng.last_transfer()
            if pack == "0":
                want = 0
            elif name == "pinned":
                want = (n - n * int(pct) // 100) & ~63
                want = n if want >= n - 64 else want
            else:
                want = n
            assert x["packed_pairs"] == want, (name, x)
            assert x["link_bytes"] == 8 * n + 2 * want + 8 * (n - want), (name, x)
        # the resident candidate list into a misaligned pageable pair of arrays
        eng.candidates(5)
        out = (np.empty(a.shape[0] + 1, np.int32)[1:], np.empty(a.shape[0], np.int32))
        eng.score_candidates(out=out)
        np.testing.assert_array_equal(out[0], cfg2_ref[0])
        np.testing.assert_array_equal(out[1], cfg2_ref[1])
        # bad pairs: (-1, -1) at their positions, every other pair scored
        bad = b.copy()
        pos = [0, 7, 8, len(bad) // 2, len(bad) - 1]
        bad[pos] = len(reads) + 5
        out = (np.empty(len(a), np.int32), np.empty(len(a), np.int32))
        with pytest.raises(OvlError, match="OVL_E_INDEX"):
            eng.score(a, bad, out=out)
        want_s, want_e = cfg2_ref[0].copy(), cfg2_ref[1].copy()
        want_s[pos] = -1
        want_e[pos] = -1
        np.testing.assert_array_equal(out[0], want_s)
        np.testing.assert_array_equal(out[1], want_e)
    finally:
        eng.close()


@pytest.mark.parametrize("scoring", [(10, -1), (1, -1), (2, 2), (-1, 3), (5, -7)])
def test_packed_chunks_scorings(oracle_mod, cfg2, scoring):
    """Packed chunks (2 bytes per pair, expanded by host threads after each chunk): cfg2's list tiled six times
    (731 K pairs) with bad pairs, under scorings with match == mismatch and mismatch > match, into pinned, pageable
    and misaligned arrays, all packed and with a direct share, twice each; every (score, end) equals the oracle's,
    and the call's link bytes are 2 per packed pair."""
    pack = "1"
    from ovlgraph import OvlError
    from ovlgraph.hostmem import pinned_empty
    reads, a0, b0 = cfg2
    match, mismatch = scoring
    rs0, re0 = oracle_mod.batch_ungapped(reads, a0, b0, match, mismatch)
    a, b = np.tile(a0, 6), np.tile(b0, 6)
    ref_s, ref_e = np.tile(rs0, 6), np.tile(re0, 6)
    n = a.shape[0] - 5
    bad = np.array([0, 63, 64, 1000, n // 2, n - 1])
    b = b.copy()
    b[bad] = len(reads) + 3
    ref_s, ref_e = ref_s.copy(), ref_e.copy()
    ref_s[bad] = ref_e[bad] = -1
    for pct in ("0", "25"):
        eng = _engine_env({"OVL_PACK": pack, "OVL_PACK_DIRECT_PCT": pct, "OVL_PAIRS_FORM": "plain"})
        try:
            eng.set_reads(reads)
            outs = {"pinned": (pinned_empty(n), pinned_empty(n)),
                    "pageable": (np.empty(n, np.int32), np.empty(n, np.int32)),
                    "misaligned": (np.empty(n + 1, np.int32)[1:], np.empty(n + 3, np.int32)[3:])}
            for name, out in outs.items():
                for rep in range(2):  # (the second call reuses the staging slots)
                    out[0][:] = 7
                    out[1][:] = 7
                    with pytest.raises(OvlError, match="OVL_E_INDEX"):
                        eng.score(a[:n], b[:n], match, mismatch, out=out)
                    np.testing.assert_array_equal(out[0], ref_s[:n], err_msg=f"{name} pct {pct} rep {rep}")
                    np.testing.assert_array_equal(out[1], ref_e[:n], err_msg=f"{name} pct {pct} rep {rep}")
                    x = eng.last_transfer()
                    np_ = x["packed_pairs"]
                    assert np_ > 0 and x["link_bytes"] == 8 * n + x["result_bytes"], x
                    res = x["result_bytes"] - 8 * (n - np_)  # the packed part's result bytes
                    assert res == 2 * np_ and x["record_pairs"] == 0, (name, x)
        finally:
            eng.close()


def test_packed_across_read_sets(oracle_mod):
    """Packed results over many calls of one engine: cfg2 and cfg3 alternating, each scored as listed (the compact
    list read in place), permuted (decoded) and from the resident candidate list, twice each, every call exact
    against the oracle (the staging slots and the heavy tiles reused across read sets)."""
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    sets = {}
    for cfg in ("cfg2", "cfg3"):
        reads, _ = dedup_reads(config_reads(cfg, seed=0))
        a, b = enumerate_candidates(reads, 5)
        rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
        sets[cfg] = (reads, a, b, rs, re_, np.random.default_rng(1).permutation(a.shape[0]))
    with _engine_env({"OVL_RESIDENT": "0"}) as eng:
        for rnd in range(2):
            for cfg in ("cfg2", "cfg3"):
                reads, a, b, rs, re_, perm = sets[cfg]
                eng.set_reads(reads)
                eng.candidates(5)
                for name in ("listed", "perm", "resident"):
                    for it in range(2):
                        if name == "resident":
                            sc, en = eng.score_candidates()
                            ws, we = rs, re_
                        elif name == "listed":
                            sc, en = eng.score(a, b)
                            ws, we = rs, re_
                        else:
                            sc, en = eng.score(a[perm], b[perm])
                            ws, we = rs[perm], re_[perm]
                        np.testing.assert_array_equal(sc, ws, err_msg=f"{rnd} {cfg} {name} {it}")
                        np.testing.assert_array_equal(en, we, err_msg=f"{rnd} {cfg} {name} {it}")
                        assert eng.last_transfer()["packed_pairs"] > 0


def test_packed_adaptive_share(oracle_mod, cfg2, cfg2_ref):
    """The direct share of 2-byte packed calls into pinned arrays (OVL_PACK=1) adapts call by call (no
    OVL_PACK_DIRECT_PCT): every call's results stay exact and the packed part stays within its bounds (50-98 % of
    the pairs)."""
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = cfg2
    eng = _engine_env({"OVL_PACK_MIN": "0", "OVL_PACK": "1", "OVL_RESIDENT": "0"})
    try:
        eng.set_reads(reads)
        eng.candidates(5)
        n = a.shape[0]
        out = (pinned_empty(n), pinned_empty(n))
        shares = []
        for _ in range(30):
            out[0][:] = -9
            eng.score_candidates(out=out)
            np.testing.assert_array_equal(out[0], cfg2_ref[0])
            np.testing.assert_array_equal(out[1], cfg2_ref[1])
            shares.append(eng.last_transfer()["packed_pairs"] / n)
        assert all(0.49 <= x <= 0.99 for x in shares), shares
    finally:
        eng.close()


@pytest.mark.parametrize("l", [254, 255])
@pytest.mark.parametrize("scoring", [(10, -1), (1, -1), (2, 2), (-1, 3), (5, -7)])
def test_packed_results_at_the_length_limit(oracle_mod, l, scoring):
    """The packed transport carries (end, mismatch count) for reads up to 254 bases (255 falls back to
    int32 results), under any scores with int32 keys: match == mismatch (mismatch count immaterial),
    mismatch > match, and pairs whose best end lies past a shorter read a (the score travels separately).
    Identical full-length reads end at l."""
    match, mismatch = scoring
    rng = np.random.default_rng(l * 10 + match)
    pack_env = {"OVL_PACK_MIN": "0"}
    base = ["".join(rng.choice(list("ACGT"), l)) for _ in range(40)]
    reads = base + [r[i + 1:] for i, r in enumerate(base[:20])]  # suffixes: a inside b's window (end > n)
    reads += [r[: l - 1 - i] for i, r in enumerate(base[20:])]  # prefixes
    m = len(reads)
    a = np.concatenate([np.arange(40), np.arange(40, 60), rng.integers(0, m, 3000)]).astype(np.int32)
    b = np.concatenate([np.arange(40), np.arange(20), rng.integers(0, m, 3000)]).astype(np.int32)
    eng = _engine_env(pack_env)
    try:
        eng.set_reads(reads)
        out = (np.empty(len(a), np.int32), np.empty(len(a), np.int32))
        eng.score(a, b, match, mismatch, out=out)
        rs, re_ = oracle_mod.batch_ungapped(reads, a, b, match, mismatch)
        np.testing.assert_array_equal(out[0], rs)
        np.testing.assert_array_equal(out[1], re_)
        if match > max(mismatch, 0):
            assert out[1][:40].tolist() == [l] * 40 and out[0][:40].tolist() == [match * l] * 40
    finally:
        eng.close()


def test_pipeline_gapped_and_banded(oracle_mod, cfg2):
    """The pipeline around the DP kernels (lane kernel above 65,536 pairs) and the band knob."""
    reads, a, b = cfg2
    eng = _engine_env({"OVL_PIPE_CHUNK": "40000"})
    try:
        eng.set_reads(reads)
        sc, en = eng.score(a, b, 10, -1, -2)
        rs, re_ = oracle_mod.batch_dp(reads, a, b, 10, -1, -2)
        np.testing.assert_array_equal(sc, rs)
        np.testing.assert_array_equal(en, re_)
        sc, en = eng.score(a, b, 10, -1, -2, 8)
        rs, re_ = oracle_mod.batch_banded(reads, a, b, 10, -1, -2, 8)
        np.testing.assert_array_equal(sc, rs)
        np.testing.assert_array_equal(en, re_)
    finally:
        eng.close()


def test_pipeline_index_error_then_recovery(engine, cfg2, cfg2_ref):
    from ovlgraph import OvlError
    reads, a, b = cfg2
    engine.set_reads(reads)
    bad = b.copy()
    bad[len(bad) // 2] = len(reads)  # one index past the read set, in the middle of a chunk
    with pytest.raises(OvlError, match="OVL_E_INDEX"):
        engine.score(a, bad)
    sc, en = engine.score(a, b)  # the flag was consumed: the next call is clean
    np.testing.assert_array_equal(sc, cfg2_ref[0])
    np.testing.assert_array_equal(en, cfg2_ref[1])
    # the kernels store the flag into pinned host memory: pageable outputs (staged copies), the gapped
    # lane kernel and the band knob report it the same way, and a clean call follows each
    pageable = (np.empty(len(a), np.int32), np.empty(len(a), np.int32))
    for args in ((10, -1, -(2 ** 31), -1), (10, -1, -2, -1), (10, -1, -2, 8)):
        with pytest.raises(OvlError, match="OVL_E_INDEX"):
            engine.score(a, bad, *args, out=pageable)
        sc, en = engine.score(a, b, *args, out=pageable)
        assert sc[len(bad) // 2] >= 0
    engine.check_device_errors()  # the device API's own flag never saw these


def test_pipeline_timing(engine, cfg2):
    reads, a, b = cfg2
    engine.set_reads(reads)
    engine.set_timing(True)
    engine.score(a, b)
    t = engine.last_timing()
    engine.set_timing(False)
    assert 0.0 < t["kernel_ms"] < t["call_ms"]


def test_registered_host_memory_is_used_in_place(engine, cfg2, cfg2_ref):
    """Results land in an ovl_host_register'ed (pinned) slice of an ordinary buffer."""
    from ovlgraph import _lib
    reads, a, b = cfg2
    engine.set_reads(reads)
    n = a.shape[0]
    L = _lib.load()
    buf = np.zeros(2 * n + 4096, np.int32)
    base = buf.ctypes.data
    _lib.check(L.ovl_host_register(ctypes.c_void_p(base), buf.nbytes))
    try:
        engine.score(a, b, out=(buf[:n], buf[n:2 * n]))
    finally:
        _lib.check(L.ovl_host_unregister(ctypes.c_void_p(base)))
    np.testing.assert_array_equal(buf[:n], cfg2_ref[0])
    np.testing.assert_array_equal(buf[n:2 * n], cfg2_ref[1])


def test_multi_device_context(oracle_mod, cfg2, cfg2_ref):
    """ovl_create(0) = every visible GPU (one on a 1-GPU box); same results as a one-GPU engine,
    through the host list and the resident device list."""
    from ovlgraph import OverlapEngine, OvlError, _lib
    reads, a, b = cfg2
    import torch
    n_dev = torch.cuda.device_count()
    eng = OverlapEngine(devices="all")
    try:
        assert eng.devices == list(range(n_dev))
        eng.set_reads(reads)
        sc, en = eng.score(a, b)
        np.testing.assert_array_equal(sc, cfg2_ref[0])
        np.testing.assert_array_equal(en, cfg2_ref[1])
        assert eng.enumerate_candidates(5) == a.shape[0]
        cs, ce = eng.score_candidates()
        np.testing.assert_array_equal(cs, cfg2_ref[0])
        np.testing.assert_array_equal(ce, cfg2_ref[1])
    finally:
        eng.close()
    with pytest.raises(OvlError, match="OVL_E_ARG"):
        OverlapEngine(devices=[0, 0])
    with pytest.raises(OvlError, match="OVL_E_ARG"):
        OverlapEngine(devices=[n_dev])
    ctx = ctypes.c_void_p()
    L = _lib.load()
    assert L.ovl_create(n_dev + 1, ctypes.byref(ctx)) == -1


@pytest.mark.parametrize("slots", [2, 3])
@pytest.mark.parametrize("chunk", ["20000", "0"])
def test_multi_device_sharding_on_shared_gpu(oracle_mod, cfg2, cfg2_ref, slots, chunk):
    """N-device contexts with every slot on GPU 0 (OVL_SHARE_DEVICES=1): the Σ n·m shards of host and
    device lists, per-device kernels and their slices of pinned / pageable results, the gapped and banded
    kernels storing through host mappings, in 20,000-pair pipeline chunks and in the automatic ones."""
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = cfg2
    eng = _engine_env({"OVL_SHARE_DEVICES": "1", "OVL_PIPE_CHUNK": chunk},
                      devices=[0] * slots)
    try:
        assert eng.devices == [0] * slots
        eng.set_reads(reads)
        n = a.shape[0]
        sc, en = eng.score(a, b)
        np.testing.assert_array_equal(sc, cfg2_ref[0])
        np.testing.assert_array_equal(en, cfg2_ref[1])
        out = (np.full(n, 7, np.int32), np.full(n, 7, np.int32))
        pa, pb = pinned_empty(n), pinned_empty(n)
        pa[:], pb[:] = a, b
        eng.score(pa, pb, out=out)
        np.testing.assert_array_equal(out[0], cfg2_ref[0])
        np.testing.assert_array_equal(out[1], cfg2_ref[1])
        assert eng.enumerate_candidates(5) == n
        cs, ce = eng.score_candidates()
        np.testing.assert_array_equal(cs, cfg2_ref[0])
        np.testing.assert_array_equal(ce, cfg2_ref[1])
        cs, ce = eng.score_candidates_range(1000, n - 777, out=(out[0][:n - 1777], out[1][:n - 1777]))
        np.testing.assert_array_equal(cs, cfg2_ref[0][1000:n - 777])
        for args, ref in (((10, -1, -2), oracle_mod.batch_dp), ((10, -1, -2, 8), oracle_mod.batch_banded)):
            idx = np.arange(0, n, 7)
            sc, en = eng.score(a[idx], b[idx], *args)
            rs, re_ = ref(reads, a[idx], b[idx], *args)
            np.testing.assert_array_equal(sc, rs)
            np.testing.assert_array_equal(en, re_)
        bad = b.copy()
        bad[-3] = len(reads)  # in the last shard
        from ovlgraph import OvlError
        with pytest.raises(OvlError, match="OVL_E_INDEX"):
            eng.score(a, bad)
        sc, en = eng.score(a, b)
        np.testing.assert_array_equal(sc, cfg2_ref[0])
    finally:
        eng.close()


def test_device_count_rule(cfg2):
    """ovl_devices_for: a host-array call uses several of a context's devices only from 3 of them with >= 262,144
    pairs each, else one (the single-device paths: packed results, the resident grid), so a context over every GPU
    is never slower than one GPU; a context whose slots share the GPU (tests) still shards every call."""
    from ovlgraph.hostmem import pinned_empty
    reads, a, b = cfg2
    for slots, cases in ((1, {10: 1, 5_000_000: 1}),
                         (2, {100_000: 1, 5_000_000: 1}),
                         (3, {100_000: 1, 786_431: 1, 786_432: 3, 5_000_000: 3}),
                         (8, {600_000: 1, 1_000_000: 3, 2_000_000: 7, 2_097_152: 8, 50_000_000: 8})):
        eng = _engine_env({"OVL_SHARE_DEVICES": "1"}, devices=[0] * slots)
        try:
            for n, want in cases.items():
                assert eng.devices_for(n) == want, (slots, n)
            if slots == 3:  # (shared slots: every call still sharded -- exact over the 3 device workers)
                eng.set_reads(reads)
                n = a.shape[0]
                out = (pinned_empty(n), pinned_empty(n))
                eng.score(a, b, out=out)
                assert eng.resident_stats()["launches"] == 0
        finally:
            eng.close()


def test_contexts_on_concurrent_host_threads(oracle_mod, cfg2, cfg2_ref):
    """Separate contexts are independent (include/ovl.h): four Python threads (ctypes releases the GIL)
    score through their own engines at once, with pageable arrays, so the staging copies of all calls
    share the process's copy pool."""
    import threading
    from ovlgraph import OverlapEngine
    reads, a, b = cfg2
    n = a.shape[0]
    errors, results = [], {}
    # (engines made here, one at a time: _engine_env sets and restores os.environ, which threads would race on
    # and could leave set for later tests)
    engines = [_engine_env({"OVL_PIPE_CHUNK": str(9000 + 1000 * t)}) for t in range(4)]
    assert "OVL_PIPE_CHUNK" not in os.environ

    def work(t):
        try:
            eng = engines[t]
            try:
                eng.set_reads(reads)
                for rep in range(5):
                    out = (np.empty(n, np.int32), np.empty(n, np.int32))
                    if (t + rep) % 2:
                        eng.score(a, b, out=out)
                    else:
                        eng.enumerate_candidates(5)
                        eng.score_candidates(out=out)
                    results[(t, rep)] = out
            finally:
                eng.close()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors
    assert len(results) == 20
    for out in results.values():
        np.testing.assert_array_equal(out[0], cfg2_ref[0])
        np.testing.assert_array_equal(out[1], cfg2_ref[1])
    assert OverlapEngine  # the engines above were independent contexts on GPU 0


def test_device_shard_bounds_and_ranges(engine, cfg2, cfg2_ref):
    from ovlgraph.sharded import pair_costs, shard_bounds
    reads, a, b = cfg2
    engine.set_reads(reads)
    n = engine.enumerate_candidates(5)
    cost = pair_costs(reads, a, b)
    for shards in (1, 2, 3, 8):
        bounds = engine.candidate_shards(shards)
        want = [0] + [shard_bounds(n, shards, r, cost)[1] for r in range(shards)]
        assert bounds == want
        parts = [engine.score_candidates_range(bounds[r], bounds[r + 1]) for r in range(shards)]
        np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), cfg2_ref[0])
        np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), cfg2_ref[1])
    sc, en = engine.score_candidates_range(10, 10)
    assert sc.size == 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_world1():
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def test_sharded_paths_on_rccl_world1(nccl_world1, engine, cfg2, cfg2_ref):
    """The multi-process drop-in's GPU branches: RCCL world 1, real engine."""
    from ovlgraph.sharded import ShardedStep, score_pairs_sharded
    reads, a, b = cfg2
    sc, en = score_pairs_sharded(reads, a, b, engine=engine)
    np.testing.assert_array_equal(sc, cfg2_ref[0])
    np.testing.assert_array_equal(en, cfg2_ref[1])
    for dest in ("host", "rank0"):
        for kw in ({"a_idx": a, "b_idx": b}, {"k": 5}):
            st = ShardedStep(reads, engine=engine, dest=dest, **kw)
            st.step()
            st.step()
            got = st.results()
            st.close()
            np.testing.assert_array_equal(got[0], cfg2_ref[0])
            np.testing.assert_array_equal(got[1], cfg2_ref[1])
    # gapped and banded scoring through the same steps (bench.py's sharded cfg5 band sweep), two buffers alive
    keep = ShardedStep(reads, engine=engine, dest="host", k=5)
    for band in (8, -1):
        engine.set_reads(reads)
        engine.enumerate_candidates(5)
        ref = engine.score_candidates(10, -1, -2, band)
        for dest in ("host", "rank0"):
            st = ShardedStep(reads, engine=engine, dest=dest, k=5, indel=-2, band=band)
            st.step()
            got = st.results()
            st.close()
            np.testing.assert_array_equal(got[0], ref[0])
            np.testing.assert_array_equal(got[1], ref[1])
    keep.close()
    # packed results (OVL_PACK_MIN=0: below the default threshold) expanded into the registered shared buffer
    packed = _engine_env({"OVL_PACK_MIN": "0"})
    try:
        st = ShardedStep(reads, engine=packed, dest="host", k=5)
        st.step()
        st.step()
        assert packed.last_transfer()["packed_pairs"] > 0
        got = st.results()
        st.close()
        np.testing.assert_array_equal(got[0], cfg2_ref[0])
        np.testing.assert_array_equal(got[1], cfg2_ref[1])
    finally:
        packed.close()


def test_lane_kernel_on_two_streams(oracle_mod, cfg2):
    """dp_lane_kernel launches on different streams are ordered on the shared hand-off buffer."""
    import torch
    reads, a, b = cfg2
    eng = _engine_env({"OVL_DP_FORM": "lane"})
    try:
        eng.set_reads(reads)
        ta = torch.as_tensor(a, device="cuda")
        tb = torch.as_tensor(b, device="cuda")
        outs = []
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for _ in range(3):
            for s in streams:
                so = torch.empty_like(ta)
                eo = torch.empty_like(ta)
                eng.score_tensors(ta, tb, so, eo, 10, -1, -2, stream=s)
                outs.append((so, eo))
        torch.cuda.synchronize()
        eng.check_device_errors()
        rs, re_ = oracle_mod.batch_dp(reads, a, b, 10, -1, -2)
        for so, eo in outs:
            np.testing.assert_array_equal(so.cpu().numpy(), rs)
            np.testing.assert_array_equal(eo.cpu().numpy(), re_)
    finally:
        eng.close()


# ----------------------------------------------------------------------------- cfg5 at full size

@pytest.fixture(scope="module")
def cfg5():
    from ovlgraph.candidates import dedup_reads, enumerate_candidates
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads("cfg5", seed=0))
    a, b = enumerate_candidates(reads, 5)
    return reads, a, b


def test_cfg5_full_default_scoring_vs_oracle(engine, oracle_mod, cfg5):
    """Every one of cfg5's pairs (default scoring: the W = 8 uniform sweep) == the oracle."""
    reads, a, b = cfg5
    assert a.shape[0] > 3_000_000
    engine.set_reads(reads)
    assert engine.plan() == "ungapped"
    sc, en = engine.score(a, b)
    rs, re_ = oracle_mod.batch_ungapped(reads, a, b)
    np.testing.assert_array_equal(sc, rs)
    np.testing.assert_array_equal(en, re_)
    n = engine.enumerate_candidates(5)
    assert n == a.shape[0]
    cs, ce = engine.score_candidates()
    np.testing.assert_array_equal(cs, rs)
    np.testing.assert_array_equal(ce, re_)


def test_cfg5_full_gapped_lane_vs_wavefront_and_oracle(oracle_mod, cfg5):
    """Gapped (indel -2) on the whole cfg5 list: the lane-per-pair full DP (the planner's choice, here
    dp_lane_h2_kernel: two pairs per lane in packed f16) == dp_fast_kernel (OVL_DP_FORM=fast) pair for pair;
    both == the oracle's full DP on a strided 50k-pair sample."""
    reads, a, b = cfg5
    lane = _engine_env({"OVL_DP_FORM": "lane"})
    fast = _engine_env({"OVL_DP_FORM": "fast"})
    try:
        lane.set_reads(reads)
        fast.set_reads(reads)
        ls, le = lane.score(a, b, 10, -1, -2)
        fs, fe = fast.score(a, b, 10, -1, -2)
    finally:
        lane.close()
        fast.close()
    np.testing.assert_array_equal(ls, fs)
    np.testing.assert_array_equal(le, fe)
    idx = np.linspace(0, a.shape[0] - 1, 50_000).astype(np.int64)
    rs, re_ = oracle_mod.batch_dp(reads, a[idx], b[idx], 10, -1, -2)
    np.testing.assert_array_equal(ls[idx], rs)
    np.testing.assert_array_equal(le[idx], re_)


# ----------------------------------------------------------------------------- the step's transport
@pytest.mark.parametrize("cfg", ["target", "cfg3"])
@pytest.mark.parametrize("pct", [None, "15"])
def test_step_transport_vs_oracle(oracle_mod, cfg, pct):
    """Whole resident list into pinned arrays through the bench step's transport (packed chunks of 2 bytes per pair
    expanded by host threads, the last pairs stored as int32 straight into the arrays; the share adaptive or fixed
    by OVL_PACK_DIRECT_PCT) equals the oracle call after call, into reused and fresh arrays; ovl_last_transfer
    counts 2 B per packed pair and 8 B per direct pair."""
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.hostmem import pinned_empty
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    env = {"OVL_RESIDENT": "0"}  # (the launch transport; the resident grid: test_gpu_resident.py)
    if pct:
        env["OVL_PACK_DIRECT_PCT"] = pct
    eng = _engine_env(env)
    try:
        eng.set_reads(reads)
        a, b = eng.candidates(5)
        ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b)
        n = a.shape[0]
        out = (pinned_empty(n), pinned_empty(n))
        for it in range(6):
            out[0][:] = -7
            out[1][:] = -7
            eng.score_candidates(out=out)
            np.testing.assert_array_equal(out[0], ref_s, err_msg=f"call {it}")
            np.testing.assert_array_equal(out[1], ref_e, err_msg=f"call {it}")
            x = eng.last_transfer()
            assert 0 < x["packed_pairs"] < n, x
            # (no pair list crosses: the link bytes are the results', 2 B per packed and 8 B per direct pair)
            assert x["link_bytes"] == x["result_bytes"], x
            assert x["result_bytes"] == 2 * x["packed_pairs"] + 8 * (n - x["packed_pairs"]), x
            assert x["record_pairs"] == 0, x
        fresh = eng.score_candidates()
        np.testing.assert_array_equal(fresh[0], ref_s)
        np.testing.assert_array_equal(fresh[1], ref_e)
    finally:
        eng.close()


def test_heavy_tiles_follow_the_list(oracle_mod):
    """Heavy tiles (tiles holding a side pair, scheduled first) are rebuilt for every new list, also when the
    new list has the same length: two read sets with the same count and different length mixes at k = 0
    (n (n - 1) pairs each), then a set with no side pairs at all."""
    from ovlgraph.hostmem import pinned_empty
    rng = np.random.default_rng(5)
    n_reads, lw = 700, 100

    def reads_with(short_at):
        rs = ["".join(rng.choice(list("ACGT"), lw)) for _ in range(n_reads)]
        for i in short_at:
            rs[i] = rs[i][: int(rng.integers(10, lw))]
        return rs

    sets = [reads_with([3, 50, 51, 400]), reads_with([10, 600, 699]), reads_with([])]
    eng = _engine_env({})
    try:
        for rs in sets:
            eng.set_reads(rs)
            a, b = eng.candidates(0)
            assert a.shape[0] == n_reads * (n_reads - 1)
            ref_s, ref_e = oracle_mod.batch_closed_form(rs, a, b)
            out = (pinned_empty(a.shape[0]), pinned_empty(a.shape[0]))
            for _ in range(2):
                eng.score_candidates(out=out)
                np.testing.assert_array_equal(out[0], ref_s)
                np.testing.assert_array_equal(out[1], ref_e)
    finally:
        eng.close()

"""GPU: the resident scoring grid (ovl_kernels.hip resident_kernel, ovl_resident.h) against the oracle.

With OVL_RESIDENT=1 (opt-in), ovl_score_candidates(_range) calls of the uniform kernel's form go to a kernel that
stays on the device between calls and takes requests through pinned memory.  Every result is compared bit for bit with the
oracle's closed form (oracle/ovl_oracle.c, the restatement of aligners.py:27-57 where gaps cannot win), call after
call: into reused and fresh, pinned and pageable, aligned and misaligned arrays; over shards that start inside a
tile, enough calls for the record ring to wrap many laps; after the grid left by itself (idle) or was asked to
(ovl_quiesce, other entry points), through close and reopen, with two contexts on one thread and with another
thread's grid on the device (that context falls back to the launch pipeline).
"""
import os
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine(env=None):
    """A context with the resident grid on (OVL_RESIDENT=1: opt-in, the default is the launch pipeline)."""
    from ovlgraph import OverlapEngine
    env = {"OVL_RESIDENT": "1", **(env or {})}
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


def _setup(cfg):
    from ovlgraph.candidates import dedup_reads
    from ovlgraph.reads import config_reads
    reads, _ = dedup_reads(config_reads(cfg, seed=0))
    return reads


@pytest.fixture(scope="module")
def cfg2_case(oracle_mod):
    reads = _setup("cfg2")
    with _engine() as eng:
        eng.set_reads(reads)
        a, b = eng.candidates(5)
    a, b = np.array(a), np.array(b)
    return reads, a, b, oracle_mod.batch_closed_form(reads, a, b)


@pytest.mark.parametrize("cfg", ["cfg2", "target", "cfg3"])
def test_resident_whole_list_call_after_call(oracle_mod, cfg):
    """The whole list, six calls into one pinned pair of arrays (poisoned between calls), then fresh arrays,
    pageable and misaligned ones: one launch serves every call; the special pairs (shorter reads a inside b's
    window) cross as ring special words."""
    from ovlgraph.hostmem import pinned_empty
    reads = _setup(cfg)
    eng = _engine()
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
        # (a gap between calls longer than the grid's idle deadline -- the checks above take ~20 ms at cfg3 -- lets
        # it leave: the next call relaunches it; never a second launch otherwise)
        st = eng.resident_stats()
        assert st["alive"] == 1 and st["launches"] == 1 + st["relaunches"] and st["broken"] == 0, st
        # back to back, no gap: one grid serves every call (after the first, which may find it gone)
        eng.score_candidates(out=out)
        before = eng.resident_stats()["launches"]
        for _ in range(20):
            eng.score_candidates(out=out)
        assert eng.resident_stats()["launches"] == before
        np.testing.assert_array_equal(out[0], ref_s)
        np.testing.assert_array_equal(out[1], ref_e)
        x = eng.last_transfer()
        assert x["record_pairs"] == n and x["result_bytes"] == 128 * ((n + 63) // 64) + 8 * x["escapes"], x
        if cfg == "target":
            assert x["escapes"] > 0, x  # (PhiX reads cut at the genome end: window pairs)
        fresh = eng.score_candidates()
        np.testing.assert_array_equal(fresh[0], ref_s)
        np.testing.assert_array_equal(fresh[1], ref_e)
        for name, o in (("pageable", (np.empty(n, np.int32), np.empty(n, np.int32))),
                        ("misaligned", (np.empty(n + 1, np.int32)[1:], np.empty(n + 3, np.int32)[3:]))):
            eng.score_candidates(out=o)
            np.testing.assert_array_equal(o[0], ref_s, err_msg=name)
            np.testing.assert_array_equal(o[1], ref_e, err_msg=name)
        # (allocating fresh arrays can take longer than the grid's idle deadline: it may have left and come back)
        st = eng.resident_stats()
        assert st["launches"] == 1 + st["relaunches"] and st["broken"] == 0, st
    finally:
        eng.close()


@pytest.mark.parametrize("form", ["1", "1x3x1x4x2", "1x4x0x4x0"])
def test_resident_shards_and_ring_laps(cfg2_case, form):
    """Shards of the list (bounds from ovl_candidates_shards, starting inside tiles) in a shuffled order, 240
    calls: the ring (2,048 tiles here) wraps ~30 laps, each request's tiles carry their lap's phase.  Forms
    (OVL_RESIDENT): the default (2 blocks per CU, software-pipelined tiles, one fence per block); 3 blocks per CU
    with one fence per wavefront; one tile at a time at 4 blocks per CU."""
    from ovlgraph.hostmem import pinned_empty
    reads, a, b, (ref_s, ref_e) = cfg2_case
    rng = np.random.default_rng(3)
    eng = _engine({"OVL_RESIDENT": form})
    try:
        eng.set_reads(reads)
        eng.enumerate_candidates(5)
        ranges = []
        for shards in (2, 3, 5, 8, 13):
            bd = eng.candidate_shards(shards)
            ranges += [(bd[r], bd[r + 1]) for r in range(shards) if bd[r + 1] > bd[r]]
        ranges += [(1, 2), (63, 64), (64, 65), (100, 100 + 64 * 7 + 5), (0, 64)]
        n = a.shape[0]
        out = (pinned_empty(n), pinned_empty(n))
        for it in range(240):
            lo, hi = ranges[int(rng.integers(len(ranges)))]
            o = (out[0][lo:hi], out[1][lo:hi])
            o[0][:] = -5
            eng.score_candidates_range(lo, hi, out=o)
            np.testing.assert_array_equal(o[0], ref_s[lo:hi], err_msg=f"{it} [{lo}, {hi})")
            np.testing.assert_array_equal(o[1], ref_e[lo:hi], err_msg=f"{it} [{lo}, {hi})")
        st = eng.resident_stats()
        assert st["broken"] == 0 and st["launches"] >= 1, st
    finally:
        eng.close()


def test_resident_relaunch_after_idle_and_quiesce(cfg2_case):
    """The grid leaves by itself after ~20 ms without a request: the next call finds it gone and relaunches it
    (the pending request served by the new grid); ovl_quiesce and other entry points (a host-list call) make it
    leave at once, and the next call launches a new one."""
    reads, a, b, (ref_s, ref_e) = cfg2_case
    eng = _engine()
    try:
        eng.set_reads(reads)
        eng.enumerate_candidates(5)

        def check(tag):
            s, e = eng.score_candidates()
            np.testing.assert_array_equal(s, ref_s, err_msg=tag)
            np.testing.assert_array_equal(e, ref_e, err_msg=tag)

        check("first")
        assert eng.resident_stats()["launches"] == 1
        time.sleep(0.08)
        check("after idle")
        st = eng.resident_stats()
        assert st["relaunches"] == 1 and st["launches"] == 2 and st["alive"] == 1, st
        eng.quiesce()
        assert eng.resident_stats()["alive"] == 0
        check("after quiesce")
        assert eng.resident_stats()["launches"] == 3
        s, e = eng.score(a[:5000], b[:5000])  # a host-list call: the launch pipeline, the grid stopped first
        np.testing.assert_array_equal(s, ref_s[:5000])
        assert eng.resident_stats()["alive"] == 0
        check("after a host-list call")
        st = eng.resident_stats()
        assert st["launches"] == 4 and st["broken"] == 0, st
    finally:
        eng.close()


@pytest.mark.parametrize("scoring", [(10, -1), (1, -1), (3, -7), (5, 5), (-2, 4), (20, -100)])
def test_resident_scorings(oracle_mod, cfg2_case, scoring):
    """Other ungapped scorings (the codes hold j and X; equal match and mismatch make X immaterial; a negative
    match makes most ends 0)."""
    reads, a, b, _ = cfg2_case
    match, mismatch = scoring
    ref_s, ref_e = oracle_mod.batch_closed_form(reads, a, b, match, mismatch)
    eng = _engine()
    try:
        eng.set_reads(reads)
        eng.enumerate_candidates(5)
        if eng.plan(match, mismatch) != "ungapped":
            pytest.skip("not the ungapped plan")
        for _ in range(2):
            s, e = eng.score_candidates(match, mismatch)
            np.testing.assert_array_equal(s, ref_s)
            np.testing.assert_array_equal(e, ref_e)
        assert eng.resident_stats()["launches"] == 1
    finally:
        eng.close()


def test_resident_contexts_close_reopen_and_threads(cfg2_case):
    """Two contexts on one thread take turns (launching one's grid stops the other's); a closed context's grid
    leaves with it; a context driven by another thread while this thread's grid is on the device scores through
    the launch pipeline (no second grid), exactly."""
    reads, a, b, (ref_s, ref_e) = cfg2_case
    e1, e2 = _engine(), _engine()
    try:
        for eng in (e1, e2):
            eng.set_reads(reads)
            eng.enumerate_candidates(5)
        for it in range(4):
            for eng in (e1, e2):
                s, e = eng.score_candidates()
                np.testing.assert_array_equal(s, ref_s, err_msg=str(it))
                np.testing.assert_array_equal(e, ref_e, err_msg=str(it))
        assert e1.resident_stats()["launches"] == 4 and e2.resident_stats()["launches"] == 4
        e2.close()
        s, e = e1.score_candidates()
        np.testing.assert_array_equal(s, ref_s)
        got = {}

        def other():
            eng = _engine()
            try:
                eng.set_reads(reads)
                eng.enumerate_candidates(5)
                got["r"] = eng.score_candidates()
                got["stats"] = eng.resident_stats()
            finally:
                eng.close()

        e1.score_candidates()  # (this thread's grid is on the device)
        t = threading.Thread(target=other)
        t.start()
        t.join(timeout=120)
        assert not t.is_alive()
        np.testing.assert_array_equal(got["r"][0], ref_s)
        np.testing.assert_array_equal(got["r"][1], ref_e)
        assert got["stats"]["launches"] == 0 and got["stats"]["broken"] == 0, got["stats"]
    finally:
        e1.close()
        e2.close()
    e3 = _engine()  # reopen
    try:
        e3.set_reads(reads)
        e3.enumerate_candidates(5)
        s, e = e3.score_candidates()
        np.testing.assert_array_equal(s, ref_s)
        np.testing.assert_array_equal(e, ref_e)
        assert e3.resident_stats()["launches"] == 1
    finally:
        e3.close()


def test_resident_off_and_timing_use_the_pipeline(cfg2_case):
    """OVL_RESIDENT=0 and the default (unset), and calls with timing on (whose launch events time the pipeline),
    never launch a grid."""
    from ovlgraph import OverlapEngine
    reads, a, b, (ref_s, ref_e) = cfg2_case
    old = os.environ.pop("OVL_RESIDENT", None)
    try:
        engines = [_engine({"OVL_RESIDENT": "0"}), OverlapEngine(0)]
    finally:
        if old is not None:
            os.environ["OVL_RESIDENT"] = old
    for eng in engines:
        try:
            eng.set_reads(reads)
            eng.enumerate_candidates(5)
            s, e = eng.score_candidates()
            np.testing.assert_array_equal(s, ref_s)
            assert eng.resident_stats()["launches"] == 0
        finally:
            eng.close()
    eng = _engine()
    try:
        eng.set_reads(reads)
        eng.enumerate_candidates(5)
        eng.set_timing(True)
        s, e = eng.score_candidates()
        np.testing.assert_array_equal(e, ref_e)
        assert eng.resident_stats()["launches"] == 0 and len(eng.last_launches()) > 0
    finally:
        eng.close()

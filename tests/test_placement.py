"""Host logic without a GPU: the process-wide engine's device placement (engine.placement) and the
oracle's optimised closed form (bench.py's second CPU baseline) against its plain restatement."""
import numpy as np
import pytest

from ovlgraph import OvlError
from ovlgraph.engine import placement


def test_placement_env_priority():
    assert placement(8, {"OVL_DEVICES": "all", "OVL_DEVICE": "3", "LOCAL_RANK": "5"}) == "all"
    assert placement(8, {"OVL_DEVICES": "1,2, 7"}) == [1, 2, 7]
    assert placement(8, {"OVL_DEVICE": "3", "LOCAL_RANK": "5"}) == 3
    assert placement(8, {"LOCAL_RANK": "5"}) == 5
    assert placement(4, {"LOCAL_RANK": "6"}) == 2
    assert placement(1, {"LOCAL_RANK": "6"}) == 0


def test_placement_round_robin_by_pid():
    """joblib workers (experiments.py:537, n_jobs=-1) are separate processes: pids spread them."""
    got = [placement(8, {}, pid=p) for p in range(1000, 1016)]
    assert sorted(set(got)) == list(range(8))
    assert all(got.count(d) == 2 for d in range(8))
    assert placement(1, {}, pid=12345) == 0


def test_placement_errors():
    with pytest.raises(OvlError):
        placement(0, {})
    with pytest.raises(OvlError):
        placement(2, {"OVL_DEVICE": "2"})
    with pytest.raises(OvlError):
        placement(2, {"OVL_DEVICES": "0,5"})


def test_closed_form_cpu_matches_restatement(oracle_mod, golden_default):
    """oracle_batch_closed_form (64-base popcount) == oracle_batch_ungapped == the golden vectors
    whose reads are ACGT and <= 256 bases."""
    pairs = [p for p in golden_default["pairs"]
             if set(p["s"] + p["t"]) <= set("ACGT") and len(p["s"]) <= 256 and len(p["t"]) <= 256]
    reads = []
    for p in pairs:
        reads += [p["s"], p["t"]]
    a = np.arange(0, len(reads), 2, dtype=np.int32)
    sc, en = oracle_mod.batch_closed_form(reads, a, a + 1)
    assert sc.tolist() == [p["score"] for p in pairs]
    assert en.tolist() == [p["end"] for p in pairs]
    rng = np.random.default_rng(3)
    rr = ["".join(rng.choice(list("ACGT"), size=int(rng.integers(0, 257)))) for _ in range(200)]
    x = rng.integers(0, 200, size=4000).astype(np.int32)
    y = rng.integers(0, 200, size=4000).astype(np.int32)
    for params in ((10, -1), (1, -1), (3, -7)):
        u = oracle_mod.batch_ungapped(rr, x, y, *params)
        c = oracle_mod.batch_closed_form(rr, x, y, *params)
        np.testing.assert_array_equal(u[0], c[0])
        np.testing.assert_array_equal(u[1], c[1])

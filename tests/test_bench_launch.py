"""bench.py's launcher (no GPU): --gpus N starts N ranks through torch.distributed.run as a child process,
the ranks see WORLD_SIZE = N, rank 0's line comes back on stdout, a failing rank fails the run, and --gpus
disagreeing with a launcher's WORLD_SIZE is an error."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_launch_plan():
    assert bench.launch_plan(1, {}) == "single"
    assert bench.launch_plan(4, {}) == "spawn"
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == "rank"
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == "single"
    assert bench.launch_plan(2, {"WORLD_SIZE": "4"}).startswith("error")
    assert bench.launch_plan(8, {"WORLD_SIZE": "1"}).startswith("error")
    assert bench.launch_plan(2, {"WORLD_SIZE": "x"}).startswith("error")


def test_args_defaults():
    a = bench.parse_args([])
    assert (a.gpus, a.config, a.seed) == (1, None, 0)
    with pytest.raises(SystemExit):
        bench.parse_args(["--gpus", "0"])


def _dry(n, *extra, stderr=None):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "7", "--dry-run", *extra],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    if stderr is not None:
        stderr.append(r.stderr)
    return json.loads(lines[0])


def test_n2_stages_are_bounded_and_heard():
    """the secondary N > 1 stages run under a time budget that every rank applies alike (the slowest
    rank's elapsed time, all-reduced), later stages are recorded as skipped, and a heartbeat on rank 0's stderr
    names the running stage while a long stage runs (two ranks over gloo; each stage sleeps 1.5 s, budget 2.5 s,
    a heartbeat every 0.5 s)."""
    err = []
    got = _dry(2, "--dry-run-stage-s", "1.5", "--extra-budget", "2.5", "--heartbeat", "0.5", stderr=err)
    plan = ["weak_scaling", "cfg4_strong", "cfg5_sharded_band_sweep", "single_process_all_gpus"]
    ran = [k for k in plan if got[k] is None]
    skipped = [k for k in plan if isinstance(got[k], dict) and "skipped" in got[k]]
    assert ran == plan[:2] and skipped == plan[2:], got
    assert "weak_scaling still running" in err[0] and "cfg4_strong done" in err[0], err[0][-2000:]
    # no budget pressure: every stage runs
    got = _dry(2, "--dry-run-stage-s", "0.2")
    assert all(got[k] is None for k in plan)


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_runs_n_ranks(n):
    got = _dry(n, "--config", "cfg4")
    assert (got["n_gpus"], got["world_size"], got["backend"], got["steps"], got["warmup"]) == (n, n, "gloo", 7, 5)
    assert got["dry_run"] is True and got["config"]["workload"].startswith("cfg4")


def test_n2_line_is_the_sharded_target_list():
    """at N > 1 the line's value is the north_star target list sharded over the ranks (strong
    scaling against the N = 1 line's list), with the same-run one-GPU time, parity flag, rank 0's roofline and
    the gather used; the weak shape, cfg4 pair-sharded and the cfg5 band sweep sharded ride beside it."""
    got = _dry(2)
    assert got["metric"] == bench.METRIC and got["unit"] == "overlap-pairs/s" and got["scaling"] == "strong"
    assert got["config"]["workload"].startswith("target: PhiX N=50000 l=100")
    assert "pair-sharded x2" in got["config"]["parallelism"]
    for k in ("value", "ms_per_step", "one_gpu_ms_per_step", "speedup_vs_one_gpu", "matches_one_gpu", "roofline",
              "in_step_kernels", "step_roofline", "per_rank_ms_per_step", "rccl_gather", "cpu_baseline"):
        assert k in got, k
    assert got["gather"]["dest"] == "host" and got["gather"]["fence"] == "shm"
    assert set(("weak_scaling", "cfg4_strong", "cfg5_sharded_band_sweep", "single_process_all_gpus")) <= set(got)
    # the secondary shapes are skipped with --no-extra, and a cfg4 run does not repeat cfg4 beside itself
    assert not set(("weak_scaling", "cfg4_strong")) & set(_dry(2, "--no-extra"))
    assert "cfg4_strong" not in _dry(2, "--config", "cfg4")


def test_n1_and_n2_lines_share_metric_and_workload():
    a = bench.parse_args([])
    line = bench.multi_line(a, 1, {}, {}, {})
    assert line["scaling"] == "strong" and line["config"]["workload"].startswith("target:")


def test_failing_rank_fails_the_run():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--dry-run-fail-rank", "1"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode != 0


def test_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="4", RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr


def test_committed_profiles_on_the_line():
    """The committed profiles bench.py puts on its line (no GPU): every cfg5 band-sweep point's kernel counters
    (profiles/r05_cfg5_pmc.json) and the per-rank projections of the target list and of cfg4
    (profiles/r06_shard_steps.json, profiles/r05_cfg4_shard_steps.json) load and are in range."""
    for band in (4, 8, 16, 32, 64, -1):
        p = bench.band_pmc(band)
        assert p is not None, band
        assert 0.0 < p["valu_isa_frac"] <= 1.2 and 0.0 < p["waves_per_simd"] <= 8.0, p
        assert p["lds_bank_conflict_frac"] is not None and 0.0 <= p["lds_bank_conflict_frac"] <= 1.0, p
        assert ("dp_lane" if band < 0 else "band_lane") in p["kernel"] and p["rocprof_kernel_ms"] > 0
    assert bench.band_pmc(12345) is None
    for name in ("target", "cfg4"):
        pr = bench.per_rank_projection(name)
        assert pr is not None and pr["source"].startswith("profiles/r0"), name
        sp = pr["projected_speedup"]
        assert sp[1] == 1.0 and 1.0 < sp[2] < sp[4] < sp[8] <= 8.0, sp

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
    assert (a.gpus, a.config, a.scaling, a.seed) == (1, None, "weak", 0)
    with pytest.raises(SystemExit):
        bench.parse_args(["--gpus", "0"])


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_runs_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--config", "cfg4", "--steps", "7", "--dry-run"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # one JSON line, from rank 0 only
    got = json.loads(lines[0])
    assert got == {"n_gpus": n, "world_size": n, "backend": "gloo", "config": "cfg4", "scaling": "weak",
                   "steps": 7, "warmup": 5}


def test_failing_rank_fails_the_run():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--dry-run-fail-rank", "1"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode != 0


def test_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="4", RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr

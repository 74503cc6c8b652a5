"""bench.py's multi-process line on the one-GPU box: the N > 1 code path run at world size 1 over RCCL
(--dist-path), so its collectives (all_gather of the per-rank times), the in-step rooflines, the weak-scaling
line and the strong-scaling cfg4 shard (ShardedStep into rank 0's shared pinned buffer, checked against one
GPU scoring the whole list) all run for real; and the strong line on its own."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

BENCH = os.path.join(ROOT, "bench.py")


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dist-path", *args], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_weak_line_over_rccl_world1():
    d = _run("--config", "cfg2", "--steps", "5", "--warmup", "1")
    assert d["n_gpus"] == 1 and d["world_size"] == 1 and d["backend"] == "nccl" and d["scaling"] == "weak"
    assert d["config"]["pairs_per_rank"] == [d["config"]["pairs"]] and d["value"] > 0
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    assert d["in_step_kernels"] and d["step_roofline"]["frac"] > 0
    s = d["cfg4_strong_scaling"]
    assert s["matches_one_gpu"] is True and s["pairs"] > 30_000_000 and s["speedup_vs_one_gpu"] > 0


def test_strong_line_over_rccl_world1():
    d = _run("--config", "cfg2", "--scaling", "strong", "--steps", "5", "--warmup", "1")
    assert d["scaling"] == "strong" and d["world_size"] == 1 and d["matches_one_gpu"] is True
    assert d["one_gpu_ms_per_step"] > 0 and d["value"] > 0

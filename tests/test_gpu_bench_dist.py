"""bench.py's multi-process line on the one-GPU box: the N > 1 code path run at world size 1 over RCCL
(--dist-path), so its collectives (all_gather of the per-rank times), the in-step rooflines, the weak-scaling
line and the strong-scaling cfg4 shard (ShardedStep into rank 0's shared pinned buffer, checked against one
GPU scoring the whole list) all run for real."""
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


def test_sharded_line_over_rccl_world1():
    """The N > 1 line at world 1: the sharded list (one shard = the whole list) through ShardedStep and its step
    fence, the RCCL gather variant, and every secondary shape, each checked against one GPU."""
    d = _run("--config", "cfg2", "--steps", "5", "--warmup", "1")
    assert d["n_gpus"] == 1 and d["world_size"] == 1 and d["backend"] == "nccl" and d["scaling"] == "strong"
    assert d["matches_one_gpu"] is True and d["one_gpu_ms_per_step"] > 0 and d["value"] > 0
    assert d["config"]["pairs_per_rank"] == [d["config"]["pairs"]]
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1 and "traffic_source" in d["roofline"]
    assert d["in_step_kernels"] and d["step_roofline"]["frac"] > 0
    assert d["rccl_gather"]["matches_one_gpu"] is True and d["rccl_gather"]["backend"] == "nccl"
    assert d["weak_scaling"]["pairs_per_rank"] and d["weak_scaling"]["value"] > 0
    s = d["cfg4_strong"]
    assert s["matches_one_gpu"] is True and s["pairs"] > 30_000_000 and s["speedup_vs_one_gpu"] > 0
    sw = d["cfg5_sharded_band_sweep"]
    assert [p["band"] for p in sw["points"]] == [4, 8, 16, 32, 64, -1]
    assert all(p["matches_single_gpu"] is True for p in sw["points"])
    assert d["single_process_all_gpus"]["matches_single_gpu"] is True

"""Multi-GPU scoring: one process per GPU, candidate pairs sharded contiguously.

SURVEY.md §8e: pairs are independent, so each rank scores a contiguous range
of the ordered candidate list with no exchange during compute.  The only
collective is the final gather of ``(score, end)`` (8 bytes per pair) so the
caller sees the reference's order; on GPUs it is an RCCL ``all_gather`` over
xGMI (backend "nccl" is RCCL on ROCm), on CPU test runs it is gloo.

Every rank enumerates the same candidate list deterministically, so the read
set and pair list need no broadcast.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Tuple

import numpy as np

from .engine import INDEL_DEFAULT, OverlapEngine


def shard_bounds(n_pairs: int, world: int, rank: int, cost: Optional[np.ndarray] = None) -> Tuple[int, int]:
    """Contiguous [lo, hi) of rank `rank`; balanced by per-pair `cost` (e.g. n*m) when given."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    if cost is None or n_pairs == 0:
        return (n_pairs * rank) // world, (n_pairs * (rank + 1)) // world
    c = np.cumsum(np.asarray(cost, dtype=np.float64))
    total = c[-1]
    cuts = [0] + [int(np.searchsorted(c, total * r / world, side="left")) for r in range(1, world)] + [n_pairs]
    cuts = np.maximum.accumulate(np.minimum(cuts, n_pairs))
    return int(cuts[rank]), int(cuts[rank + 1])


def score_pairs_sharded(reads: Sequence[str], a_idx, b_idx, match: int = 10, mismatch: int = -1,
                        indel: int = INDEL_DEFAULT, group=None, engine: Optional[OverlapEngine] = None,
                        local_scorer: Optional[Callable] = None, balance: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """Score the whole pair list across the ranks of `group`; every rank gets all results.

    ``local_scorer(reads, a, b) -> (score, end)`` overrides the GPU engine for
    the local shard (used by CPU multi-process tests with the oracle).
    """
    import torch
    import torch.distributed as dist

    a = np.ascontiguousarray(a_idx, dtype=np.int32)
    b = np.ascontiguousarray(b_idx, dtype=np.int32)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cost = None
    if balance and a.shape[0]:
        lens = np.fromiter((len(r) for r in reads), dtype=np.int64, count=len(reads))
        cost = lens[a] * lens[b] + 1
    bounds = [shard_bounds(a.shape[0], world, r, cost) for r in range(world)]
    lo, hi = bounds[rank]
    width = max(h - l for l, h in bounds) if bounds else 0
    backend = dist.get_backend(group)
    on_gpu = backend == "nccl"
    device = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")

    packed = torch.full((2, max(width, 1)), -1, dtype=torch.int32, device=device)
    if hi > lo:
        if local_scorer is not None:
            sc, en = local_scorer(reads, a[lo:hi], b[lo:hi])
            packed[0, : hi - lo] = torch.as_tensor(np.asarray(sc, dtype=np.int32), device=device)
            packed[1, : hi - lo] = torch.as_tensor(np.asarray(en, dtype=np.int32), device=device)
        elif on_gpu:
            eng = engine or OverlapEngine(-1)
            eng.set_reads(reads)
            ta = torch.as_tensor(a[lo:hi], device=device)
            tb = torch.as_tensor(b[lo:hi], device=device)
            eng.score_tensors(ta, tb, packed[0], packed[1], match, mismatch, indel)
        else:
            eng = engine or OverlapEngine(-1)
            eng.set_reads(reads)
            sc, en = eng.score(a[lo:hi], b[lo:hi], match, mismatch, indel)
            packed[0, : hi - lo] = torch.as_tensor(sc)
            packed[1, : hi - lo] = torch.as_tensor(en)
    gathered = [torch.empty_like(packed) for _ in range(world)]
    dist.all_gather(gathered, packed, group=group)
    score = np.empty(a.shape[0], dtype=np.int32)
    end = np.empty(a.shape[0], dtype=np.int32)
    for r, (l, h) in enumerate(bounds):
        g = gathered[r].cpu().numpy()
        score[l:h] = g[0, : h - l]
        end[l:h] = g[1, : h - l]
    return score, end


class ShardedStep:
    """Repeated sharded scoring of one candidate list with the RCCL gather, device-resident.

    The same contract as ``score_pairs_sharded`` (every rank holds the same ordered list, each scores
    its contiguous shard, one ``all_gather`` restores reference order), split into a one-time setup
    and a ``step()`` that issues the shard's scoring launch and the gather with no host copies: the
    shard's indices and the packed ``(score, end)`` rows stay in HBM.  ``bench.py`` times it at N > 1.
    On the gloo backend (CPU tests, one-GPU rehearsal) the gather runs on host copies, and
    ``local_scorer(reads, a, b) -> (score, end)`` may replace the engine.
    """

    def __init__(self, reads: Sequence[str], a_idx, b_idx, match: int = 10, mismatch: int = -1,
                 indel: int = INDEL_DEFAULT, group=None, engine: Optional[OverlapEngine] = None,
                 local_scorer: Optional[Callable] = None, balance: bool = True):
        import torch
        import torch.distributed as dist

        self.reads = reads
        self.a = np.ascontiguousarray(a_idx, dtype=np.int32)
        self.b = np.ascontiguousarray(b_idx, dtype=np.int32)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        cost = None
        if balance and self.a.shape[0]:
            lens = np.fromiter((len(r) for r in reads), dtype=np.int64, count=len(reads))
            cost = lens[self.a] * lens[self.b] + 1
        self.bounds = [shard_bounds(self.a.shape[0], self.world, r, cost) for r in range(self.world)]
        self.width = max(1, max(h - l for l, h in self.bounds))
        self.on_gpu = dist.get_backend(group) == "nccl"
        self.local_scorer = local_scorer
        self.scoring = (match, mismatch, indel)
        lo, hi = self.bounds[self.rank]
        self.n_local = hi - lo
        self._launch = None
        if local_scorer is None:
            dev = torch.device("cuda", torch.cuda.current_device())
            self.eng = engine or OverlapEngine(dev.index)
            self.eng.set_reads(reads)
            self.packed = torch.full((2, self.width), -1, dtype=torch.int32, device=dev)
            if self.n_local:
                self.ta = torch.as_tensor(self.a[lo:hi], device=dev)
                self.tb = torch.as_tensor(self.b[lo:hi], device=dev)
                self._launch = self.eng.launcher(self.ta, self.tb, self.packed[0], self.packed[1],
                                                 match, mismatch, indel)
        else:
            self.packed = torch.full((2, self.width), -1, dtype=torch.int32)
        gdev = self.packed.device if self.on_gpu else torch.device("cpu")
        self.out = torch.empty((self.world, 2, self.width), dtype=torch.int32, device=gdev)

    def step(self) -> None:
        """Score this rank's shard, then gather every shard (asynchronous on the GPU path)."""
        import torch
        import torch.distributed as dist

        if self._launch is not None:
            self._launch()
        elif self.local_scorer is not None and self.n_local:
            lo, hi = self.bounds[self.rank]
            sc, en = self.local_scorer(self.reads, self.a[lo:hi], self.b[lo:hi])
            self.packed[0, :hi - lo] = torch.as_tensor(np.asarray(sc, dtype=np.int32))
            self.packed[1, :hi - lo] = torch.as_tensor(np.asarray(en, dtype=np.int32))
        if self.on_gpu:
            dist.all_gather_into_tensor(self.out.view(-1), self.packed.view(-1), group=self.group)
        else:
            dist.all_gather(list(self.out.unbind(0)), self.packed.cpu(), group=self.group)

    def gather_bytes(self) -> int:
        """Bytes every rank receives per step (the padded (score, end) rows of all shards)."""
        return int(self.out.numel()) * 4

    def results(self) -> Tuple[np.ndarray, np.ndarray]:
        """(score, end) of the whole list in reference order, from the last step's gather."""
        g = self.out.cpu().numpy()
        score = np.empty(self.a.shape[0], dtype=np.int32)
        end = np.empty(self.a.shape[0], dtype=np.int32)
        for r, (l, h) in enumerate(self.bounds):
            score[l:h] = g[r, 0, : h - l]
            end[l:h] = g[r, 1, : h - l]
        return score, end

"""Multi-process multi-GPU scoring: one process per GPU, candidate pairs sharded contiguously.

SURVEY.md §8e: pairs are independent, so each rank scores a contiguous range of
the ordered candidate list (balanced by Σ len(a)·len(b)) with no exchange during
compute.  The results are gathered to ONE destination, in reference order:

* ``dest="host"`` (the default of ``ShardedStep``): every rank's kernels store its
  ``(score, end)`` slice straight into a shared host buffer that rank 0 owns (POSIX
  shared memory, pinned per rank with ``ovl_host_register``).  Each GPU uses its own
  PCIe link, so the slices land in parallel; no collective moves data, and a step
  fence of a few cache lines in the buffer's header orders the steps (rank 0 waits
  for every rank's published step number).  This is SURVEY.md §8e's "per-device D2H
  into pinned host slices".
* ``dest="rank0"``: the slices stay in HBM and one ``dist.gather`` (RCCL
  send/recv over xGMI on backend "nccl", gloo on CPU) collects them on rank 0's GPU.

The single-process form of the same thing is ``OverlapEngine(devices=...)``: one
context drives every GPU and the per-device copies land in the caller's arrays.

Every rank enumerates (or receives) the same candidate list deterministically, so
the read set and pair list need no broadcast.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .engine import INDEL_DEFAULT, OverlapEngine


def shard_bounds(n_pairs: int, world: int, rank: int, cost: Optional[np.ndarray] = None) -> Tuple[int, int]:
    """Contiguous [lo, hi) of rank `rank`; balanced by per-pair `cost` (e.g. n*m + 1) when given.

    Cut r is the first pair p whose inclusive cost prefix c[p] satisfies c[p]·world >= total·r,
    the rule ``ovl_candidates_shards`` applies on the device.
    """
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    if cost is None or n_pairs == 0:
        return (n_pairs * rank) // world, (n_pairs * (rank + 1)) // world
    c = np.cumsum(np.asarray(cost, dtype=np.int64))
    total = int(c[-1])
    cuts = [0] + [int(np.searchsorted(c * world, total * r, side="left")) for r in range(1, world)] + [n_pairs]
    cuts = np.maximum.accumulate(np.minimum(cuts, n_pairs))
    return int(cuts[rank]), int(cuts[rank + 1])


def pair_costs(reads: Sequence[str], a: np.ndarray, b: np.ndarray) -> np.ndarray:
    lens = np.fromiter((len(r) for r in reads), dtype=np.int64, count=len(reads))
    return lens[a] * lens[b] + 1


def _device(dist, group):
    import torch
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _gather_rows(packed, bounds, n_pairs: int, dst: Optional[int], group):
    """Gather every rank's padded (2, width) rows to `dst` (None: to every rank) -> (score, end) or None."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if dst is None:
        rows = [torch.empty_like(packed) for _ in range(world)]
        dist.all_gather(rows, packed, group=group)
    else:
        rows = [torch.empty_like(packed) for _ in range(world)] if rank == dst else None
        dist.gather(packed, rows, dst=dst, group=group)
        if rank != dst:
            return None
    score = np.empty(n_pairs, dtype=np.int32)
    end = np.empty(n_pairs, dtype=np.int32)
    for r, (lo, hi) in enumerate(bounds):
        g = rows[r].cpu().numpy()
        score[lo:hi] = g[0, : hi - lo]
        end[lo:hi] = g[1, : hi - lo]
    return score, end


def score_pairs_sharded(reads: Sequence[str], a_idx, b_idx, match: int = 10, mismatch: int = -1,
                        indel: int = INDEL_DEFAULT, group=None, engine: Optional[OverlapEngine] = None,
                        local_scorer: Optional[Callable] = None, balance: bool = True, dst: Optional[int] = 0):
    """Score the whole pair list across the ranks of `group`; results gathered to rank `dst`.

    Returns ``(score, end)`` in reference order on rank ``dst`` and ``None`` on the others
    (``dst=None``: every rank gets them, an all_gather).  ``local_scorer(reads, a, b) ->
    (score, end)`` overrides the GPU engine for the local shard (CPU multi-process tests).
    """
    import torch
    import torch.distributed as dist

    a = np.ascontiguousarray(a_idx, dtype=np.int32)
    b = np.ascontiguousarray(b_idx, dtype=np.int32)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    cost = pair_costs(reads, a, b) if balance and a.shape[0] else None
    bounds = [shard_bounds(a.shape[0], world, r, cost) for r in range(world)]
    lo, hi = bounds[rank]
    width = max(1, max(h - l for l, h in bounds))
    device = _device(dist, group)
    packed = torch.full((2, width), -1, dtype=torch.int32, device=device)
    if hi > lo:
        if local_scorer is not None:
            sc, en = local_scorer(reads, a[lo:hi], b[lo:hi])
        else:
            eng = engine or OverlapEngine(torch.cuda.current_device() if device.type == "cuda" else -1)
            eng.set_reads(reads)
            sc, en = eng.score(a[lo:hi], b[lo:hi], match, mismatch, indel)
        packed[0, : hi - lo] = torch.as_tensor(np.asarray(sc, dtype=np.int32)).to(device)
        packed[1, : hi - lo] = torch.as_tensor(np.asarray(en, dtype=np.int32)).to(device)
    return _gather_rows(packed, bounds, a.shape[0], dst, group)


_shm_seq = 0


class SharedResults:
    """(score, end) host buffers of n pairs shared by the ranks of one node (POSIX shm).

    Rank 0 creates it, the others attach by name; each rank pins only the pages of its own
    slices (``ovl_host_register``), so its GPU's stores land in place.  ``slots`` copies of the two
    columns (each column padded to whole pages, so no two ranges share a page): step k writes
    slot k % slots.  A header page ahead of them holds the step fence (``publish`` / ``wait_all`` /
    ``release`` / ``wait_released``): one int64 counter per rank, each on its own 64-byte line and
    written by that rank only, plus rank 0's release counter.  ``score`` / ``end`` are slot 0.
    """

    LINE = 64
    PAGE = 4096
    TIMEOUT_S = 300.0

    def __init__(self, n_pairs: int, group=None, tag: str = "", slots: int = 1):
        import torch.distributed as dist
        from multiprocessing import resource_tracker, shared_memory

        global _shm_seq
        self.n = int(n_pairs)
        self.slots = max(1, int(slots))
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.hdr_bytes = -(-self.LINE * (self.world + 1) // self.PAGE) * self.PAGE
        self.col = -(-max(4, 4 * self.n) // self.PAGE) * self.PAGE // 4  # int32 per column, whole pages
        size = self.hdr_bytes + 8 * self.col * self.slots
        _shm_seq += 1  # several buffers may be alive at once (one per ShardedStep)
        name = [f"ovl_{os.getpid()}_{_shm_seq}_{tag}"[:30] if self.rank == 0 else None]
        if self.rank == 0:
            self.shm = shared_memory.SharedMemory(name=name[0], create=True, size=size)
            self.shm.buf[: self.hdr_bytes] = bytes(self.hdr_bytes)
        dist.broadcast_object_list(name, src=0, group=group)
        if self.rank != 0:
            self.shm = shared_memory.SharedMemory(name=name[0], create=False)
            # an attaching process must not unlink the segment at exit (CPython < 3.13 tracker)
            try:
                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
        stride = self.LINE // 8
        self.hdr = np.frombuffer(self.shm.buf, dtype=np.int64, count=self.hdr_bytes // 8)
        self.done = self.hdr[: stride * self.world: stride]  # done[r]: the last step rank r published
        self.released = self.hdr[stride * self.world: stride * self.world + 1]  # rank 0: last step consumed
        self.buf = np.frombuffer(self.shm.buf, dtype=np.int32, count=2 * self.col * self.slots,
                                 offset=self.hdr_bytes)
        self.score, self.end = self.slot(0)
        self._pinned: List[int] = []

    def slot(self, s: int) -> Tuple[np.ndarray, np.ndarray]:
        """(score, end) arrays of slot s."""
        o = 2 * self.col * s
        return self.buf[o: o + self.n], self.buf[o + self.col: o + self.col + self.n]

    # ---- the step fence: no collective, a few cache lines of shared host memory
    def publish(self, step: int) -> None:
        """This rank's slice of `step` is in the buffer (its scoring call has returned)."""
        self.done[self.rank] = step

    def _spin(self, ready, what: str) -> None:
        import time
        if ready():
            return
        t0 = time.perf_counter()
        spins = 0
        while not ready():
            spins += 1
            if spins > 2000:  # ~a few hundred microseconds of tight polling, then yield the CPU
                time.sleep(20e-6)
                if time.perf_counter() - t0 > self.TIMEOUT_S:
                    raise RuntimeError(f"shared results: timed out waiting for {what} "
                                       f"(done={self.done.tolist()}, released={int(self.released[0])})")

    def wait_all(self, step: int) -> None:
        """Rank 0: until every rank has published `step` (every slice has landed)."""
        self._spin(lambda: int(self.done.min()) >= step, f"every rank's step {step}")

    def release(self, step: int) -> None:
        """Rank 0: it is done reading the results of `step`; ranks may overwrite them."""
        self.released[0] = step

    def wait_released(self, step: int) -> None:
        """Ranks > 0: until rank 0 has released `step` (before writing over its results)."""
        self._spin(lambda: int(self.released[0]) >= step, f"rank 0 to release step {step}")

    def pin(self, lo: int, hi: int) -> None:
        """Pin the pages that hold pairs [lo, hi) of both columns of every slot in this process."""
        if hi <= lo:
            return
        from . import _lib
        L = _lib.load()
        base = self.buf.ctypes.data
        page = self.PAGE
        for c in range(2 * self.slots):
            first, last = c * self.col + lo, c * self.col + hi
            s = (base + 4 * first) // page * page
            e = -(-(base + 4 * last) // page) * page
            s = max(s, base + 4 * c * self.col)  # (columns start on pages: no page of another column)
            rc = L.ovl_host_register(ctypes.c_void_p(s), e - s)
            if rc != 0:
                raise _lib.OvlError(rc, _lib.last_error())
            self._pinned.append(s)

    def close(self) -> None:
        from . import _lib
        if self._pinned:
            L = _lib.load()
            for s in self._pinned:
                L.ovl_host_unregister(ctypes.c_void_p(s))
            self._pinned = []
        self.score = self.end = self.buf = self.hdr = self.done = self.released = None
        try:
            self.shm.close()
        except BufferError:
            return
        if self.rank == 0:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass


class ShardedStep:
    """Repeated sharded scoring of one candidate list, results gathered to one destination.

    Setup once: the read set on this rank's GPU, the candidate list (``a_idx``/``b_idx`` host
    arrays, or ``k`` to enumerate it on the device, identical on every rank), this rank's
    Σ n·m-balanced shard, the scoring (``match``, ``mismatch``, ``indel``, ``band``) and the
    destination.  ``step()`` scores the shard and gathers:

    * ``dest="host"``: the shard's results land in rank 0's shared host arrays (the kernels
      store into the rank's pinned slice).  On rank 0 ``step()`` returns once every slice of
      this step has landed; on the other ranks once their own slice has.  The order comes from
      the step fence in the buffer's header page (``fence="shm"``, the default): each rank
      publishes its step number after its call returns, rank 0 waits for all of them, and step k
      goes to result slot k % ``slots``, which a rank writes only after rank 0 is done reading
      step k - ``slots`` (it has called step k - ``slots`` + 1).  With two slots (the default) a
      rank may score step k while rank 0 still waits for a slower rank's step k - 1, so one
      rank's late step does not hold every other rank at the next one; every step's results are
      still complete in rank 0's buffer when its ``step()`` returns.  No collective runs per step.  ``fence="barrier"`` puts a ``dist.barrier`` after
      every step instead (the round-3 form; a barrier over RCCL costs tens of microseconds,
      about what a shard of the target list takes to score at N = 8);
    * ``dest="rank0"``: the shard's results stay in HBM and ``dist.gather`` collects them on
      rank 0 (RCCL send/recv on "nccl").

    ``results()`` gives rank 0 the reference-ordered ``(score, end)``.  On CPU tests
    ``local_scorer(reads, a, b) -> (score, end)`` replaces the engine (host lists only).
    """

    def __init__(self, reads: Sequence[str], a_idx=None, b_idx=None, k: Optional[int] = None,
                 match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT, group=None,
                 engine: Optional[OverlapEngine] = None, local_scorer: Optional[Callable] = None,
                 dest: str = "host", balance: bool = True, band: int = -1, fence: str = "shm",
                 slots: int = 2):
        import torch
        import torch.distributed as dist

        if dest not in ("host", "rank0"):
            raise ValueError("dest must be 'host' or 'rank0'")
        if fence not in ("shm", "barrier"):
            raise ValueError("fence must be 'shm' or 'barrier'")
        self.fence = fence
        self.steps = 0
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dest = dest
        self.scoring = (match, mismatch, indel, band)
        self.local_scorer = local_scorer
        self.reads = reads
        self.device = _device(dist, group)
        self.eng = None
        self.a = self.b = None
        if local_scorer is None:
            self.eng = engine or OverlapEngine(torch.cuda.current_device())
            self.eng.set_reads(reads)
        if a_idx is None:
            if self.eng is None or k is None:
                raise ValueError("give a_idx/b_idx, or k with the GPU engine")
            n = self.eng.enumerate_candidates(k)
            self.n_pairs = n
            cuts = self.eng.candidate_shards(self.world) if balance else \
                [(n * r) // self.world for r in range(self.world + 1)]
            self.bounds = [(cuts[r], cuts[r + 1]) for r in range(self.world)]
            self.on_device_list = True
        else:
            self.a = np.ascontiguousarray(a_idx, dtype=np.int32)
            self.b = np.ascontiguousarray(b_idx, dtype=np.int32)
            self.n_pairs = int(self.a.shape[0])
            cost = pair_costs(reads, self.a, self.b) if balance and self.n_pairs else None
            self.bounds = [shard_bounds(self.n_pairs, self.world, r, cost) for r in range(self.world)]
            self.on_device_list = False
        lo, hi = self.bounds[self.rank]
        self.lo, self.hi = lo, hi
        self.width = max(1, max(h - l for l, h in self.bounds))
        self.shared = None
        self._launch = None
        self._launches = []
        if dest == "host":
            self.shared = SharedResults(self.n_pairs, group, tag=str(os.environ.get("MASTER_PORT", "")),
                                        slots=slots if fence == "shm" else 1)
            if self.eng is not None:
                self.shared.pin(lo, hi)
                if self.on_device_list and hi > lo:
                    # one foreign call per step (ctypes arguments converted once), one per result slot
                    for sl in range(self.shared.slots):
                        sc, en = self.shared.slot(sl)
                        self._launches.append(self.eng.range_scorer(lo, hi, (sc[lo:hi], en[lo:hi]),
                                                                    match, mismatch, indel, band))
                    self._launch = self._launches[0]
        else:
            self.packed = torch.full((2, self.width), -1, dtype=torch.int32, device=self.device)
            self.rows = ([torch.empty_like(self.packed) for _ in range(self.world)] if self.rank == 0 else None)
            if self.eng is not None and hi > lo and self.device.type != "cuda":
                # gloo (one-GPU rehearsal): the rows live in host memory, so score through the host API
                rows = self.packed.numpy()
                if self.on_device_list:
                    self._launch = lambda: self.eng.score_candidates_range(
                        lo, hi, match, mismatch, indel, band, out=(rows[0], rows[1]))
                else:
                    self._launch = lambda: self.eng.score(self.a[lo:hi], self.b[lo:hi], match, mismatch, indel,
                                                          band, out=(rows[0], rows[1]))
            elif self.eng is not None and hi > lo:
                if self.on_device_list:
                    pa, pb, _ = self.eng.candidates_device()
                    self._launch = lambda: self.eng.score_device(
                        pa + 4 * lo, pb + 4 * lo, hi - lo, self.packed[0].data_ptr(), self.packed[1].data_ptr(),
                        match, mismatch, indel, band, stream=torch.cuda.current_stream(self.device).cuda_stream)
                else:
                    self.ta = torch.as_tensor(self.a[lo:hi], device=self.device)
                    self.tb = torch.as_tensor(self.b[lo:hi], device=self.device)
                    self._launch = self.eng.launcher(self.ta, self.tb, self.packed[0], self.packed[1],
                                                     match, mismatch, indel, band)

    def _local(self):
        lo, hi = self.lo, self.hi
        return self.local_scorer(self.reads, self.a[lo:hi], self.b[lo:hi])

    def step(self) -> None:
        """Score this rank's shard and gather it to the destination."""
        import torch
        import torch.distributed as dist

        lo, hi = self.lo, self.hi
        if self.dest == "host":
            self.steps += 1
            k = self.steps
            sl = k % self.shared.slots
            if self.fence == "shm":
                if self.rank == 0:
                    self.shared.release(k - 1)  # rank 0 is done with step k - 1's results
                else:
                    self.shared.wait_released(k - self.shared.slots)  # (slot sl last held that step)
            if self._launches:
                self._launches[sl]()
            elif hi > lo:
                sc, en = self.shared.slot(sl)
                out = (sc[lo:hi], en[lo:hi])
                if self.eng is None:
                    sc, en = self._local()
                    out[0][:] = sc
                    out[1][:] = en
                else:
                    self.eng.score(self.a[lo:hi], self.b[lo:hi], *self.scoring, out=out)
            if self.fence == "barrier":
                dist.barrier(group=self.group)
                return
            self.shared.publish(k)
            if self.rank == 0:
                self.shared.wait_all(k)
            return
        if self._launch is not None:
            self._launch()
        elif self.eng is None and hi > lo:
            sc, en = self._local()
            self.packed[0, : hi - lo] = torch.as_tensor(np.asarray(sc, dtype=np.int32))
            self.packed[1, : hi - lo] = torch.as_tensor(np.asarray(en, dtype=np.int32))
        dist.gather(self.packed, self.rows, dst=0, group=self.group)

    def gather_bytes(self) -> int:
        """Result bytes that cross to the destination per step (8 B per pair; padded rows for rank0)."""
        if self.dest == "host":
            return 8 * self.n_pairs
        return self.world * 2 * self.width * 4

    def results(self) -> Optional[Tuple[np.ndarray, np.ndarray]]:
        """Rank 0: (score, end) of the whole list in reference order, from the last step; else None."""
        if self.rank != 0:
            return None
        if self.dest == "host":
            sc, en = self.shared.slot(self.steps % self.shared.slots)
            return sc.copy(), en.copy()
        score = np.empty(self.n_pairs, dtype=np.int32)
        end = np.empty(self.n_pairs, dtype=np.int32)
        for r, (l, h) in enumerate(self.bounds):
            g = self.rows[r].cpu().numpy()
            score[l:h] = g[0, : h - l]
            end[l:h] = g[1, : h - l]
        return score, end

    def close(self) -> None:
        import torch.distributed as dist
        self._launch = None  # (these hold views of the shared buffer)
        self._launches = []
        if self.shared is not None:
            if self.fence == "shm" and self.rank == 0:
                self.shared.release(self.steps)
            dist.barrier(group=self.group)  # rank 0 unlinks only after every rank is done
            self.shared.close()
            self.shared = None

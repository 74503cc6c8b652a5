"""OverlapEngine — Python face of libovl.so (one context on one or more GPUs).

The engine keeps a read set resident in HBM (bit-plane packed by a gfx950
kernel) and scores candidate pairs in one batched call, replacing the
per-pair Python->Numba call of overlapGraphs.py:53.  A multi-GPU engine
(``OverlapEngine(devices=[...])`` or ``devices="all"``) shards every host-array
call over its GPUs from this one thread.  Results come back in
pinned host arrays (``hostmem.PinnedPool``) unless ``out=`` is given.  It never
computes on the CPU: a missing library or GPU raises ``OvlError``.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from ._lib import OvlError, check
from .hostmem import pinned_empty

INDEL_DEFAULT = -(2 ** 31)  # aligners.py:7 default indel (the report's "-inf", REPORT p.3)

_LIVE: "weakref.WeakSet[OverlapEngine]" = weakref.WeakSet()  # open contexts (quiesce_all)


def quiesce_all() -> None:
    """ovl_quiesce on every open context of this process: their resident scoring grids leave the device, so a
    whole-device synchronisation (torch.cuda.synchronize) that follows does not wait for the grids' idle deadline.
    Call it from the thread that drives the contexts."""
    for eng in list(_LIVE):
        if getattr(eng, "_ctx", None):
            eng.quiesce()


def encode_reads(reads: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    """Concatenate reads into one byte buffer + int64 offsets.

    Bytes are symbols compared for equality only, so any injective
    character->byte map preserves the reference's ``s[i-1] == t[j-1]`` test
    (aligners.py:35).  Latin-1 covers every str whose characters are < 256;
    otherwise up to 256 distinct characters are renumbered.
    """
    n = len(reads)
    offs = np.zeros(n + 1, dtype=np.int64)
    if n:
        np.cumsum(np.fromiter((len(r) for r in reads), dtype=np.int64, count=n), out=offs[1:])
    joined = "".join(reads)
    try:
        buf = np.frombuffer(joined.encode("latin-1"), dtype=np.uint8)
    except UnicodeEncodeError:
        table: Dict[str, int] = {}
        for ch in joined:
            if ch not in table:
                if len(table) >= 256:
                    raise OvlError(-4, "more than 256 distinct symbols in the read set")
                table[ch] = len(table)
        buf = np.fromiter((table[ch] for ch in joined), dtype=np.uint8, count=len(joined))
    if buf.size == 0:
        buf = np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(buf), offs


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _outputs(n: int, out) -> Tuple[np.ndarray, np.ndarray]:
    """Result arrays: the caller's ``out=(score, end)`` (int32, contiguous, >= n) or pinned ones."""
    if out is None:
        return pinned_empty(n), pinned_empty(n)
    sc, en = out
    for x in (sc, en):
        if not (isinstance(x, np.ndarray) and x.dtype == np.int32 and x.flags.c_contiguous and x.ndim == 1
                and x.shape[0] >= n and x.flags.writeable):
            raise OvlError(-1, "out must be two writeable contiguous 1-D int32 arrays of >= n_pairs elements")
    return sc[:n], en[:n]


def host_pool() -> Dict[str, int]:
    """The host thread pool's plan, recounted now (ovl_host_pool): {threads, sharers, cpus, packed}."""
    v = [ctypes.c_int32() for _ in range(4)]
    check(_lib.load().ovl_host_pool(*[ctypes.byref(x) for x in v]))
    return dict(zip(("threads", "sharers", "cpus", "packed"), (x.value for x in v)))


def device_count() -> int:
    n = ctypes.c_int32(0)
    rc = _lib.load().ovl_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class OverlapEngine:
    """A libovl context on one HIP device (``device``; -1 = the current one) or on several
    (``devices``: a list of ordinals, or "all")."""

    def __init__(self, device: int = -1, devices: Union[None, str, Sequence[int]] = None):
        self._L = _lib.load()
        n = ctypes.c_int32(0)
        rc = self._L.ovl_device_count(ctypes.byref(n))
        if rc != 0 or n.value <= 0:
            raise OvlError(-2, "no HIP device visible to libovl: the overlap engine has no CPU fallback "
                               f"({_lib.last_error()})")
        ctx = ctypes.c_void_p()
        if devices == "all":
            check(self._L.ovl_create(0, ctypes.byref(ctx)))
        elif devices is not None:
            ids = np.ascontiguousarray(list(devices), dtype=np.int32)
            check(self._L.ovl_create_on_devices(_ptr(ids), int(ids.shape[0]), ctypes.byref(ctx)))
        elif int(device) < 0:
            check(self._L.ovl_create(1, ctypes.byref(ctx)))
        else:
            ids = np.array([int(device)], dtype=np.int32)
            check(self._L.ovl_create_on_devices(_ptr(ids), 1, ctypes.byref(ctx)))
        self._ctx = ctx
        self._reads_key = None
        self._dev0 = self.devices[0]  # device pointers given to score_device / score_tensors live here
        _LIVE.add(self)

    def _check_tensors(self, what: str, *ts) -> None:
        """Contiguous int32 tensors on this engine's first device (kernels there read and write them)."""
        import torch
        for t in ts:
            if t.dtype != torch.int32 or not t.is_cuda or not t.is_contiguous():
                raise OvlError(-1, f"{what} needs contiguous int32 device tensors")
            if t.device.index != self._dev0:
                raise OvlError(-1, f"{what}: tensor on cuda:{t.device.index}, but this engine's kernels run on "
                                   f"cuda:{self._dev0}")

    @property
    def devices(self) -> List[int]:
        """Device ordinals of this context (results are sharded over them in this order)."""
        n = ctypes.c_int32()
        ids = np.zeros(64, dtype=np.int32)
        check(self._L.ovl_ctx_devices(self._ctx, _ptr(ids), 64, ctypes.byref(n)), self._ctx)
        return ids[: n.value].tolist()

    def set_timing(self, on: bool = True) -> None:
        """Record kernel time inside host-array scoring calls (HIP events; see ``last_timing``)."""
        check(self._L.ovl_set_timing(self._ctx, 1 if on else 0), self._ctx)

    def last_timing(self) -> Dict[str, float]:
        """{kernel_ms: summed kernel time of the busiest device, call_ms: wall time} of the last call."""
        k, w = ctypes.c_double(), ctypes.c_double()
        check(self._L.ovl_last_timing(self._ctx, ctypes.byref(k), ctypes.byref(w)), self._ctx)
        return {"kernel_ms": k.value, "call_ms": w.value}

    def last_launches(self) -> List[Dict[str, float]]:
        """The scoring launches of the last host-array call made with timing on (ovl_last_launches):
        [{device, sink (0 HBM, 1 int32 into host memory, 2 packed into host staging), pairs, ms}]."""
        n = ctypes.c_int32()
        check(self._L.ovl_last_launches(self._ctx, 0, None, None, None, None, ctypes.byref(n)), self._ctx)
        k = n.value
        dev, sink = np.zeros(max(k, 1), np.int32), np.zeros(max(k, 1), np.int32)
        pairs, ms = np.zeros(max(k, 1), np.int64), np.zeros(max(k, 1), np.float64)
        check(self._L.ovl_last_launches(self._ctx, k, _ptr(dev), _ptr(sink), _ptr(pairs), _ptr(ms),
                                        ctypes.byref(n)), self._ctx)
        return [{"device": int(dev[i]), "sink": int(sink[i]), "pairs": int(pairs[i]), "ms": float(ms[i])}
                for i in range(min(k, n.value))]

    def last_transfer(self) -> Dict[str, int]:
        """{link_bytes, packed_pairs} of the last host-array scoring call (ovl_last_transfer) and its results'
        part: result_bytes, record_pairs (crossed as tile records), escapes (ovl_last_results)."""
        b, p = ctypes.c_int64(), ctypes.c_int64()
        check(self._L.ovl_last_transfer(self._ctx, ctypes.byref(b), ctypes.byref(p)), self._ctx)
        r, q, e = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(self._L.ovl_last_results(self._ctx, ctypes.byref(r), ctypes.byref(q), ctypes.byref(e)), self._ctx)
        return {"link_bytes": b.value, "packed_pairs": p.value, "result_bytes": r.value, "record_pairs": q.value,
                "escapes": e.value}

    def last_pair_list(self) -> Dict[str, int]:
        """{in_place_pairs, decoded_pairs} of the last host-array call (ovl_last_pair_list): how the compact
        host pair list reached the kernels (read in place by uniform_kernel, or decoded into HBM first)."""
        i, d = ctypes.c_int64(), ctypes.c_int64()
        check(self._L.ovl_last_pair_list(self._ctx, ctypes.byref(i), ctypes.byref(d)), self._ctx)
        return {"in_place_pairs": i.value, "decoded_pairs": d.value}

    # ---------------------------------------------------------------- lifecycle
    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._L.ovl_destroy(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- reads
    def set_reads(self, reads: Sequence[str], encoded: Optional[Tuple[np.ndarray, np.ndarray]] = None) -> None:
        """Upload, encode and bit-plane pack a read set; it stays resident in HBM."""
        buf, offs = encoded if encoded is not None else encode_reads(reads)
        n = offs.shape[0] - 1
        check(self._L.ovl_set_reads(self._ctx, _ptr(buf), _ptr(offs), n), self._ctx)
        self._reads_key = id(reads)

    def info(self) -> Dict[str, int]:
        n, lmax, planes = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        nbytes = ctypes.c_int64()
        check(self._L.ovl_reads_info(self._ctx, ctypes.byref(n), ctypes.byref(lmax), ctypes.byref(planes),
                                     ctypes.byref(nbytes)), self._ctx)
        return {"n_reads": n.value, "lmax": lmax.value, "planes": planes.value, "device_bytes": nbytes.value}

    def plan(self, match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT, band: int = -1) -> str:
        k = ctypes.c_int32()
        check(self._L.ovl_plan(self._ctx, match, mismatch, indel, band, ctypes.byref(k)), self._ctx)
        return _lib.KERNELS[k.value]

    # ---------------------------------------------------------------- candidates
    def candidates(self, k: int = 5) -> Tuple[np.ndarray, np.ndarray]:
        """k-mer candidate pairs over the resident (distinct) reads, enumerated on the GPU.

        Same list and order as ``candidates.enumerate_candidates`` (overlapGraphs.py:30-52);
        the list also stays resident for ``score_candidates``.
        """
        return self.candidates_copy(self.enumerate_candidates(k))

    def candidates_copy(self, n: int) -> Tuple[np.ndarray, np.ndarray]:
        """The resident candidate list (``n`` pairs, from ``enumerate_candidates``) in pinned host arrays."""
        a = pinned_empty(n)
        b = pinned_empty(n)
        if n:
            check(self._L.ovl_candidates_copy(self._ctx, _ptr(a), _ptr(b)), self._ctx)
        return a, b

    def enumerate_candidates(self, k: int = 5) -> int:
        """Enumerate the candidate list on the device (kept resident); returns its length."""
        if k < 0:
            raise AssertionError("k-mer length must be non-negative")
        n = ctypes.c_int64()
        check(self._L.ovl_candidates(self._ctx, int(k), ctypes.byref(n)), self._ctx)
        return int(n.value)

    def candidates_device(self) -> Tuple[int, int, int]:
        """(device ptr of a_idx, device ptr of b_idx, n_pairs) of the resident candidate list."""
        pa, pb, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
        check(self._L.ovl_candidates_device(self._ctx, ctypes.byref(pa), ctypes.byref(pb), ctypes.byref(n)),
              self._ctx)
        return pa.value or 0, pb.value or 0, int(n.value)

    def score_candidates(self, match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT,
                         band: int = -1, out=None) -> Tuple[np.ndarray, np.ndarray]:
        """Score the resident candidate list (no pair upload) -> (score, end) host arrays.

        Sharded over the engine's devices; each device's results land in its slice of the
        arrays by DMA (pinned arrays unless ``out=(score, end)`` is given)."""
        n = self.candidates_device()[2]
        sc, en = _outputs(n, out)
        check(self._L.ovl_score_candidates(self._ctx, match, mismatch, indel, band, _ptr(sc), _ptr(en)),
              self._ctx)
        return sc, en

    def score_candidates_range(self, lo: int, hi: int, match: int = 10, mismatch: int = -1,
                               indel: int = INDEL_DEFAULT, band: int = -1, out=None) -> Tuple[np.ndarray, np.ndarray]:
        """(score, end) of candidate pairs [lo, hi) (a shard of a multi-process job)."""
        sc, en = _outputs(int(hi) - int(lo), out)
        check(self._L.ovl_score_candidates_range(self._ctx, int(lo), int(hi), match, mismatch, indel, band,
                                                 _ptr(sc), _ptr(en)), self._ctx)
        return sc, en

    def range_scorer(self, lo: int, hi: int, out, match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT,
                     band: int = -1):
        """Pre-bound ``score_candidates_range(lo, hi, ..., out=out)`` for repeated steps over the same shard and
        arrays: every argument converted to its ctypes form once, so a step costs one foreign call (the
        sharded step of a multi-process job calls it every step).  ``out`` must stay alive while it is used."""
        sc, en = _outputs(int(hi) - int(lo), out)
        fn = self._L.ovl_score_candidates_range
        ctx = self._ctx
        args = (ctx, ctypes.c_int64(int(lo)), ctypes.c_int64(int(hi)), ctypes.c_int32(match), ctypes.c_int32(mismatch),
                ctypes.c_int64(indel), ctypes.c_int32(band), _ptr(sc), _ptr(en))
        check(self._L.ovl_plan(ctx, match, mismatch, indel, band, ctypes.byref(ctypes.c_int32())), ctx)

        keep = (self, sc, en)  # the closure owns the result arrays (and the engine) its pointers name

        def score() -> None:
            if keep[0]._ctx is None:
                raise RuntimeError("range_scorer: the engine is closed")
            rc = fn(*args)
            if rc:
                check(rc, ctx)
        return score

    def devices_for(self, n_pairs: int) -> int:
        """How many of this context's devices a host-array call over n_pairs uses (ovl_devices_for)."""
        k = ctypes.c_int32()
        check(self._L.ovl_devices_for(self._ctx, int(n_pairs), ctypes.byref(k)), self._ctx)
        return k.value

    def quiesce(self) -> None:
        """Make this context's resident scoring grids leave the device now (ovl_quiesce): before a whole-device
        synchronisation (torch.cuda.synchronize), which would otherwise wait for their idle deadline.  The next
        eligible scoring call relaunches them."""
        check(self._L.ovl_quiesce(self._ctx), self._ctx)

    def resident_stats(self) -> Dict[str, int]:
        """{alive, launches, relaunches, broken} of this context's resident grids (ovl_resident_stats)."""
        al, br = ctypes.c_int32(), ctypes.c_int32()
        ln, rl = ctypes.c_int64(), ctypes.c_int64()
        check(self._L.ovl_resident_stats(self._ctx, ctypes.byref(al), ctypes.byref(ln), ctypes.byref(rl),
                                         ctypes.byref(br)), self._ctx)
        return {"alive": al.value, "launches": ln.value, "relaunches": rl.value, "broken": br.value}

    def candidate_shards(self, n_shards: int) -> List[int]:
        """Shard bounds of the resident candidate list balanced by sum len(a)*len(b) + 1 (on the device)."""
        bounds = np.zeros(int(n_shards) + 1, dtype=np.int64)
        check(self._L.ovl_candidates_shards(self._ctx, int(n_shards), _ptr(bounds)), self._ctx)
        return bounds.tolist()

    # ---------------------------------------------------------------- local alignment
    def local_align(self, query: str, reference: str, match: int = 10, mismatch: int = -1, indel: int = -1,
                    traceback: bool = True):
        """local_alignment's DP (aligners.py:105-160) on the GPU for one (possibly large) pair.

        Returns (score, end_i, end_j, start_i, start_j, ops) with ops the walk's codes
        (1 diag, 2 up, 3 left) in walk order (None without traceback).
        """
        buf, offs = encode_reads([query, reference])
        n, m = len(query), len(reference)
        qb = np.ascontiguousarray(buf[:n]) if n else np.zeros(1, np.uint8)
        rb = np.ascontiguousarray(buf[n:n + m]) if m else np.zeros(1, np.uint8)
        outs = [ctypes.c_int32() for _ in range(5)]
        k = ctypes.c_int64()
        cap = n + m + 1
        ops = np.zeros(cap, dtype=np.int8) if traceback else None
        check(self._L.ovl_local_align(self._ctx, _ptr(qb), n, _ptr(rb), m, int(match), int(mismatch), int(indel),
                                      *[ctypes.byref(o) for o in outs], _ptr(ops) if traceback else None,
                                      cap if traceback else 0, ctypes.byref(k)), self._ctx)
        sc, ei, ej, si, sj = (o.value for o in outs)
        return sc, ei, ej, si, sj, (ops[: k.value] if traceback else None)

    # ---------------------------------------------------------------- scoring
    def score_pairs(self, reads: Sequence[str], a_idx, b_idx, match: int = 10, mismatch: int = -1,
                    indel: int = INDEL_DEFAULT, band: int = -1, out=None,
                    encoded: Optional[Tuple[np.ndarray, np.ndarray]] = None) -> Tuple[np.ndarray, np.ndarray]:
        """The one-shot ABI call ``ovl_score_pairs``: host reads + host pair list -> host
        (score, end); the reads are uploaded, packed and left resident (as ``set_reads``)."""
        buf, offs = encoded if encoded is not None else encode_reads(reads)
        a = np.ascontiguousarray(a_idx, dtype=np.int32)
        b = np.ascontiguousarray(b_idx, dtype=np.int32)
        if a.shape != b.shape or a.ndim != 1:
            raise OvlError(-1, "a_idx and b_idx must be 1-D arrays of equal length")
        sc, en = _outputs(a.shape[0], out)
        check(self._L.ovl_score_pairs(self._ctx, _ptr(buf), _ptr(offs), offs.shape[0] - 1, _ptr(a), _ptr(b),
                                      a.shape[0], match, mismatch, indel, band, _ptr(sc), _ptr(en)), self._ctx)
        self._reads_key = id(reads)
        return sc, en

    def score(self, a_idx, b_idx, match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT,
              band: int = -1, out=None) -> Tuple[np.ndarray, np.ndarray]:
        """Score pairs (host arrays) against the resident reads -> (score, end) int32 arrays
        (pinned unless ``out=(score, end)`` is given); sharded over the engine's devices."""
        a = np.ascontiguousarray(a_idx, dtype=np.int32)
        b = np.ascontiguousarray(b_idx, dtype=np.int32)
        if a.shape != b.shape or a.ndim != 1:
            raise OvlError(-1, "a_idx and b_idx must be 1-D arrays of equal length")
        sc, en = _outputs(a.shape[0], out)
        check(self._L.ovl_score_host(self._ctx, _ptr(a), _ptr(b), a.shape[0], match, mismatch, indel, band,
                                     _ptr(sc), _ptr(en)), self._ctx)
        return sc, en

    def score_device(self, a_ptr: int, b_ptr: int, n_pairs: int, score_ptr: int, end_ptr: int,
                     match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT, band: int = -1,
                     stream: int = 0) -> None:
        """Asynchronous scoring with device pointers (e.g. torch tensors' data_ptr()) on `stream`."""
        check(self._L.ovl_score_device(self._ctx, ctypes.c_void_p(a_ptr), ctypes.c_void_p(b_ptr), int(n_pairs),
                                       match, mismatch, indel, band, ctypes.c_void_p(score_ptr),
                                       ctypes.c_void_p(end_ptr), ctypes.c_void_p(stream or None)), self._ctx)

    def score_tensors(self, a, b, out_score, out_end, match: int = 10, mismatch: int = -1,
                      indel: int = INDEL_DEFAULT, band: int = -1, stream=None) -> None:
        """torch int32 device tensors in/out, launched on torch's current stream (or `stream`)."""
        import torch
        self._check_tensors("score_tensors", a, b, out_score, out_end)
        n = a.numel()
        if b.numel() != n or out_score.numel() < n or out_end.numel() < n:
            raise OvlError(-1, "tensor sizes disagree")
        s = stream if stream is not None else torch.cuda.current_stream(a.device)
        self.score_device(a.data_ptr(), b.data_ptr(), n, out_score.data_ptr(), out_end.data_ptr(),
                          match, mismatch, indel, band, stream=s.cuda_stream)

    def launcher(self, a, b, out_score, out_end, match: int = 10, mismatch: int = -1,
                 indel: int = INDEL_DEFAULT, band: int = -1, stream=None):
        """Pre-bound scoring launch for repeated steps over the same device buffers.

        Converts every argument to its ctypes form once, so each call costs one
        foreign call (the launch itself) instead of per-call tensor checks.
        The tensors must stay alive while the launcher is used.
        """
        import torch
        self._check_tensors("launcher", a, b, out_score, out_end)
        n = a.numel()
        if b.numel() != n or out_score.numel() < n or out_end.numel() < n:
            raise OvlError(-1, "tensor sizes disagree")
        s = stream if stream is not None else torch.cuda.current_stream(a.device)
        fn = self._L.ovl_score_device
        ctx = self._ctx
        args = (ctx, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_int64(n),
                ctypes.c_int32(match), ctypes.c_int32(mismatch), ctypes.c_int64(indel), ctypes.c_int32(band),
                ctypes.c_void_p(out_score.data_ptr()), ctypes.c_void_p(out_end.data_ptr()),
                ctypes.c_void_p(s.cuda_stream or None))
        check(self._L.ovl_plan(ctx, match, mismatch, indel, band, ctypes.byref(ctypes.c_int32())), ctx)

        def launch() -> None:
            rc = fn(*args)
            if rc:
                check(rc, ctx)
        return launch

    def check_device_errors(self) -> None:
        check(self._L.ovl_check_device_errors(self._ctx), self._ctx)

    def align_one(self, a: int, b: int, n: int, m: int, match: int = 10, mismatch: int = -1,
                  indel: int = INDEL_DEFAULT, traceback: bool = False):
        """One resident pair through the DP kernel; optionally the int8 traceback table."""
        sc, en = ctypes.c_int32(), ctypes.c_int32()
        tb = np.zeros((n + 1) * (m + 1), dtype=np.int8) if traceback else None
        check(self._L.ovl_align_one(self._ctx, a, b, match, mismatch, indel, ctypes.byref(sc), ctypes.byref(en),
                                    _ptr(tb) if tb is not None else None), self._ctx)
        if traceback:
            return sc.value, en.value, tb.reshape(n + 1, m + 1)
        return sc.value, en.value


_default: Optional[OverlapEngine] = None
_default_lock = threading.Lock()


def placement(count: int, env=None, pid: Optional[int] = None) -> Union[int, str, List[int]]:
    """Which device(s) the process-wide engine uses, given ``count`` visible devices.

    1. ``OVL_DEVICES``: "all" or a comma list -> one engine over several GPUs (single process);
    2. ``OVL_DEVICE``: that ordinal;
    3. ``LOCAL_RANK`` (torch.distributed.run and similar launchers): local_rank % count;
    4. otherwise the process id modulo count, so the reference's joblib workers
       (experiments.py:537, n_jobs=-1: one process each) spread over the visible GPUs.
    """
    env = os.environ if env is None else env
    if count <= 0:
        raise OvlError(-2, "no HIP device visible to libovl")
    many = env.get("OVL_DEVICES")
    if many:
        if many.strip().lower() == "all":
            return "all"
        ids = [int(x) for x in many.split(",") if x.strip()]
        if not ids or any(not 0 <= i < count for i in ids):
            raise OvlError(-1, f"OVL_DEVICES={many!r}: ordinals must lie in [0, {count})")
        return ids
    one = env.get("OVL_DEVICE")
    if one not in (None, ""):
        d = int(one)
        if not 0 <= d < count:
            raise OvlError(-1, f"OVL_DEVICE={d} outside [0, {count})")
        return d
    lr = env.get("LOCAL_RANK")
    if lr not in (None, ""):
        return int(lr) % count
    return (os.getpid() if pid is None else pid) % count


def default_engine() -> OverlapEngine:
    """Process-wide engine (created on first use) on the device(s) ``placement`` picks."""
    global _default
    with _default_lock:
        if _default is None:
            where = placement(device_count())
            if isinstance(where, int):
                _default = OverlapEngine(where)
            else:
                _default = OverlapEngine(devices=where)
        return _default


def score_reads(reads: Sequence[str], a_idx, b_idx, match: int = 10, mismatch: int = -1,
                indel: int = INDEL_DEFAULT, band: int = -1,
                engine: Optional[OverlapEngine] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Upload `reads` and score the pair list in one batch on the GPU."""
    eng = engine or default_engine()
    eng.set_reads(reads)
    return eng.score(a_idx, b_idx, match, mismatch, indel, band)

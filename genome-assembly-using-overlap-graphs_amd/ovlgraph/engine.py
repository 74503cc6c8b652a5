"""OverlapEngine — Python face of libovl.so (one context per GPU, one GPU per process).

The engine keeps a read set resident in HBM (bit-plane packed by a gfx950
kernel) and scores candidate pairs in one batched call, replacing the
per-pair Python->Numba call of overlapGraphs.py:53.  It never computes on the
CPU: a missing library or GPU raises ``OvlError``.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import OvlError, check

INDEL_DEFAULT = -(2 ** 31)  # aligners.py:7 default indel (the report's "-inf", REPORT p.3)


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


class OverlapEngine:
    """A libovl context bound to one HIP device."""

    def __init__(self, device: int = -1):
        self._L = _lib.load()
        n = ctypes.c_int32(0)
        rc = self._L.ovl_device_count(ctypes.byref(n))
        if rc != 0 or n.value <= 0:
            raise OvlError(-2, "no HIP device visible to libovl: the overlap engine has no CPU fallback "
                               f"({_lib.last_error()})")
        ctx = ctypes.c_void_p()
        check(self._L.ovl_create(int(device), ctypes.byref(ctx)))
        self._ctx = ctx
        self._reads_key = None

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
        n = self.enumerate_candidates(k)
        a = np.empty(n, dtype=np.int32)
        b = np.empty(n, dtype=np.int32)
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
                         band: int = -1) -> Tuple[np.ndarray, np.ndarray]:
        """Score the resident candidate list (no pair upload) -> (score, end) host arrays."""
        n = self.candidates_device()[2]
        sc = np.empty(n, dtype=np.int32)
        en = np.empty(n, dtype=np.int32)
        check(self._L.ovl_score_candidates(self._ctx, match, mismatch, indel, band, _ptr(sc), _ptr(en)),
              self._ctx)
        return sc, en

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
    def score(self, a_idx, b_idx, match: int = 10, mismatch: int = -1, indel: int = INDEL_DEFAULT,
              band: int = -1) -> Tuple[np.ndarray, np.ndarray]:
        """Score pairs (host arrays) against the resident reads -> (score, end) int32 arrays."""
        a = np.ascontiguousarray(a_idx, dtype=np.int32)
        b = np.ascontiguousarray(b_idx, dtype=np.int32)
        if a.shape != b.shape or a.ndim != 1:
            raise OvlError(-1, "a_idx and b_idx must be 1-D arrays of equal length")
        sc = np.empty(a.shape[0], dtype=np.int32)
        en = np.empty(a.shape[0], dtype=np.int32)
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
        for t in (a, b, out_score, out_end):
            if t.dtype != torch.int32 or not t.is_cuda or not t.is_contiguous():
                raise OvlError(-1, "score_tensors needs contiguous int32 device tensors")
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
        for t in (a, b, out_score, out_end):
            if t.dtype != torch.int32 or not t.is_cuda or not t.is_contiguous():
                raise OvlError(-1, "launcher needs contiguous int32 device tensors")
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


def default_engine() -> OverlapEngine:
    """Process-wide engine on the current HIP device (created on first use)."""
    global _default
    with _default_lock:
        if _default is None:
            _default = OverlapEngine(-1)
        return _default


def score_reads(reads: Sequence[str], a_idx, b_idx, match: int = 10, mismatch: int = -1,
                indel: int = INDEL_DEFAULT, band: int = -1,
                engine: Optional[OverlapEngine] = None) -> Tuple[np.ndarray, np.ndarray]:
    """Upload `reads` and score the pair list in one batch on the GPU."""
    eng = engine or default_engine()
    eng.set_reads(reads)
    return eng.score(a_idx, b_idx, match, mismatch, indel, band)

"""Pinned host memory for scoring results (and pair lists), handed out as numpy arrays.

A scoring call's results leave the GPU by DMA.  Into pageable numpy memory that
costs a staging copy (and, for a fresh ``np.empty``, a page fault per 4 KiB); into
pinned memory the DMA lands in place at PCIe rate (results back
in host memory).  Pinning is slow (~ms per MB-scale block), so blocks are cached
and reused, like torch's caching host allocator: ``PinnedPool.empty`` hands out a
numpy array on a cached block of the next power-of-two size, and the block returns
to the cache when the last view of that array is garbage collected.
"""
from __future__ import annotations

import ctypes
import threading
import weakref
from typing import Dict, List

import numpy as np

from . import _lib
from ._lib import check

_MIN_BLOCK = 1 << 12


class PinnedPool:
    """Caching allocator of pinned host blocks (``ovl_host_alloc``)."""

    def __init__(self, max_cached_bytes: int = 1 << 31):
        self._L = _lib.load()
        self._free: Dict[int, List[int]] = {}
        self._lock = threading.Lock()
        self._cached = 0
        self.max_cached_bytes = max_cached_bytes
        self.allocations = 0  # blocks pinned so far (diagnostics / tests)

    def _block(self, nbytes: int) -> int:
        size = max(_MIN_BLOCK, 1 << max(0, int(nbytes - 1).bit_length()))
        with self._lock:
            lst = self._free.get(size)
            if lst:
                self._cached -= size
                return lst.pop(), size
        ptr = ctypes.c_void_p()
        check(self._L.ovl_host_alloc(size, ctypes.byref(ptr)))
        self.allocations += 1
        return ptr.value, size

    def _release(self, ptr: int, size: int) -> None:
        with self._lock:
            if self._cached + size <= self.max_cached_bytes:
                self._free.setdefault(size, []).append(ptr)
                self._cached += size
                return
        self._L.ovl_host_free(ctypes.c_void_p(ptr))

    def empty(self, n: int, dtype=np.int32) -> np.ndarray:
        """A 1-D array of n elements on pinned memory (contents undefined)."""
        dt = np.dtype(dtype)
        ptr, size = self._block(max(1, n) * dt.itemsize)
        raw = (ctypes.c_char * size).from_address(ptr)
        fin = weakref.finalize(raw, self._release, ptr, size)
        fin.atexit = False  # the HIP runtime may already be gone at interpreter exit
        return np.frombuffer(raw, dtype=dt, count=n)

    def trim(self) -> None:
        """Unpin every cached block."""
        with self._lock:
            blocks = [(p, s) for s, lst in self._free.items() for p in lst]
            self._free.clear()
            self._cached = 0
        for p, _ in blocks:
            self._L.ovl_host_free(ctypes.c_void_p(p))


_pool = None
_pool_lock = threading.Lock()


def pinned_pool() -> PinnedPool:
    """The process-wide pool (created on first use)."""
    global _pool
    with _pool_lock:
        if _pool is None:
            _pool = PinnedPool()
        return _pool


def pinned_empty(n: int, dtype=np.int32) -> np.ndarray:
    return pinned_pool().empty(n, dtype)


def is_pinned_array(a: np.ndarray) -> bool:
    """True when ``a``'s memory came from the pool (its base chain ends at a pooled ctypes block)."""
    base = a
    while isinstance(base, np.ndarray) and base.base is not None:
        base = base.base
    return isinstance(base, ctypes.Array)

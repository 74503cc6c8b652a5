"""k-mer candidate-pair enumeration (host side; stays in Python per BASELINE.json north_star).

Produces exactly the ordered pair list that ``construct_overlap_graph_nx_k``
feeds to ``overlap_alignment`` in the reference (overlapGraphs.py:17-52):

* reads are de-duplicated in first-occurrence order (``read_copies``,
  overlapGraphs.py:18-20);
* for ``k > 0`` a prefix index maps ``read[:k]`` (the whole read when it is
  shorter than ``k``) to the reads carrying it, in ``read_copies`` order
  (overlapGraphs.py:30-40);
* the outer loop walks ``read_copies`` in order; its lookup key is
  ``read[-k:]`` (whole read when shorter, overlapGraphs.py:44-47); the inner
  loop walks the indexed list in order, or every distinct read when ``k == 0``
  (overlapGraphs.py:49-50); identical reads are skipped (overlapGraphs.py:52).

Indices refer to positions in the de-duplicated read list.
``enumerate_candidates`` is the vectorised version used by the product path;
``enumerate_candidates_loop`` is a literal loop restatement kept as its checker.
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Sequence, Tuple

import numpy as np


def dedup_reads(reads: Sequence[str]) -> Tuple[List[str], List[int]]:
    """Distinct reads in first-occurrence order plus their copy counts (overlapGraphs.py:18-20).

    ``Counter`` counts in C and keeps first-insertion order, the order of the reference's
    ``read_copies[read] = read_copies.get(read, 0) + 1`` loop."""
    counts = Counter(reads)
    return list(counts.keys()), list(counts.values())


def _prefix_key(r: str, k: int) -> str:
    return r[:k] if len(r) >= k else r


def _suffix_key(r: str, k: int) -> str:
    return r[-k:] if len(r) >= k > 0 else r


def enumerate_candidates_loop(distinct: Sequence[str], k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Literal restatement of overlapGraphs.py:30-52 (slow; used to check the vectorised path)."""
    if k < 0:
        raise AssertionError("k-mer length must be non-negative")
    index: Dict[str, List[int]] = {}
    if k > 0:
        for i, r in enumerate(distinct):
            index.setdefault(_prefix_key(r, k), []).append(i)
    all_idx = list(range(len(distinct)))
    a_out: List[int] = []
    b_out: List[int] = []
    for ia, ra in enumerate(distinct):
        cands = index.get(_suffix_key(ra, k), []) if k > 0 else all_idx
        for ib in cands:
            if ib != ia:  # distinct list => index inequality == string inequality
                a_out.append(ia)
                b_out.append(ib)
    return np.asarray(a_out, dtype=np.int32), np.asarray(b_out, dtype=np.int32)


def enumerate_candidates(distinct: Sequence[str], k: int) -> Tuple[np.ndarray, np.ndarray]:
    """Vectorised candidate enumeration with the reference's iteration order.

    Returns ``(a_idx, b_idx)`` int32 arrays; pair ``p`` means
    ``overlap_alignment(distinct[a_idx[p]], distinct[b_idx[p]])``.
    """
    if k < 0:
        raise AssertionError("k-mer length must be non-negative")
    D = len(distinct)
    if D == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    if k == 0:
        # every ordered pair (a, b) with a != b, a-major, b ascending
        a = np.repeat(np.arange(D, dtype=np.int64), D - 1)
        b = np.tile(np.arange(D - 1, dtype=np.int64), D)
        b = b + (b >= a)  # skip the diagonal while keeping b ascending
        return a.astype(np.int32), b.astype(np.int32)

    key_ids: Dict[str, int] = {}
    pre = np.empty(D, dtype=np.int64)
    for i, r in enumerate(distinct):
        pre[i] = key_ids.setdefault(_prefix_key(r, k), len(key_ids))
    n_keys = len(key_ids)
    suf = np.empty(D, dtype=np.int64)
    for i, r in enumerate(distinct):
        suf[i] = key_ids.get(_suffix_key(r, k), -1)

    order = np.argsort(pre, kind="stable")          # reads grouped by prefix key, index order kept
    sizes = np.bincount(pre, minlength=n_keys)
    starts = np.zeros(n_keys + 1, dtype=np.int64)
    np.cumsum(sizes, out=starts[1:])

    has = suf >= 0
    cnt = np.zeros(D, dtype=np.int64)
    cnt[has] = sizes[suf[has]]
    total = int(cnt.sum())
    if total == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    a = np.repeat(np.arange(D, dtype=np.int64), cnt)
    # position of each output inside its group: global position minus the group's first output
    first_out = np.zeros(D, dtype=np.int64)
    np.cumsum(cnt[:-1], out=first_out[1:])
    grp_start = np.zeros(D, dtype=np.int64)
    grp_start[has] = starts[suf[has]]
    pos = np.arange(total, dtype=np.int64) - np.repeat(first_out, cnt) + np.repeat(grp_start, cnt)
    b = order[pos]
    keep = a != b
    return a[keep].astype(np.int32), b[keep].astype(np.int32)

"""ORACLE — TEST INFRASTRUCTURE ONLY (parity checker, never the product).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  The product path (``ovlgraph``) never touches it.

Contents:
* ``overlap_alignment`` — pure-Python restatement of ``aligners.py:6-82``
  (fill, last-row argmax, backtrack strings and ``to_print``), with Numba's
  integer semantics: int64 arithmetic, stores wrapped to int32.  Slow: small
  cases only.
* ``ungapped`` — the closed form of SURVEY.md fact 3 (gaps can never win).
* ``gaps_cannot_win`` — the condition under which the closed form is exact.
* ``batch_dp`` / ``batch_ungapped`` — the C restatement (``ovl_oracle.c``),
  OpenMP over pairs; ``batch_dp`` is the CPU baseline timed by bench.py.
* ``graph_nx_k`` — restatement of ``overlapGraphs.py:5-61`` (node/edge order).

Pinning: checked against tests/golden/*.json, which were generated from the
reference's own source by oracle/gen_golden.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

INT32_MIN = -(2 ** 31)


def _wrap32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def overlap_alignment(s: str, t: str, match_score: int = 10, mismatch: int = -1,
                      indel: int = INT32_MIN):
    """Restatement of aligners.py:6-82 returning the same 5-tuple."""
    n, m = len(s), len(t)
    dp = [[0] * (m + 1) for _ in range(n + 1)]
    tb = [[0] * (m + 1) for _ in range(n + 1)]
    for i in range(1, n + 1):
        prev, cur, trow = dp[i - 1], dp[i], tb[i]
        si = s[i - 1]
        for j in range(1, m + 1):
            diag = prev[j - 1] + (match_score if si == t[j - 1] else mismatch)
            up = prev[j] + indel
            left = cur[j - 1] + indel
            if diag >= up and diag >= left:
                cur[j] = _wrap32(diag); trow[j] = 0
            elif up >= left:
                cur[j] = _wrap32(up); trow[j] = 1
            else:
                cur[j] = _wrap32(left); trow[j] = 2
    best, end = float("-inf"), 0
    for j in range(m + 1):
        if dp[n][j] > best:
            best, end = dp[n][j], j
    a_s: List[str] = []
    a_t: List[str] = []
    i, j = n, end
    while i > 0 and j > 0:
        d = tb[i][j]
        if d == 0:
            a_s.append(s[i - 1]); a_t.append(t[j - 1]); i -= 1; j -= 1
        elif d == 1:
            a_s.append(s[i - 1]); a_t.append("-"); i -= 1
        else:
            a_s.append("-"); a_t.append(t[j - 1]); j -= 1
    align_s = "".join(reversed(a_s))
    align_t = "".join(reversed(a_t))
    to_print = f"\nTarget:   {align_t}\n          {'|' * len(align_t)}\nQuery:    {align_s}"
    return to_print, align_s, align_t, int(best), end


def ungapped(s: str, t: str, match_score: int = 10, mismatch: int = -1) -> Tuple[int, int]:
    """Closed form: best last-row diagonal sum, first argmax."""
    n, m = len(s), len(t)
    best, end = 0, 0
    for j in range(1, m + 1):
        L = min(n, j)
        tot = 0
        for q in range(L):
            tot += match_score if s[n - L + q] == t[j - L + q] else mismatch
        if tot > best:
            best, end = tot, j
    return best, end


def gaps_cannot_win(match: int, mismatch: int, indel: int, lmax: int) -> bool:
    """True when every DP cell provably takes the diagonal branch (aligners.py:40).

    By induction every dp value is a sum of at most lmax diagonal terms, so
    diag >= min(0, lmax*min(match, mismatch)) and dp <= max(0, lmax*max(...));
    'up'/'left' add indel to a dp value, so indel <= lo - hi suffices.
    """
    lo = min(0, lmax * min(match, mismatch))
    hi = max(0, lmax * max(match, mismatch))
    return indel <= lo - hi


# ----------------------------------------------------------------------------- C oracle

def build() -> str:
    """Compile oracle/ovl_oracle.c (idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i32, i64 = ctypes.c_int32, ctypes.c_int64
        L.oracle_version.restype = ctypes.c_int
        L.oracle_overlap_dp.argtypes = [P, i32, P, i32, i64, i64, i64, P, P, P]
        L.oracle_overlap_dp.restype = ctypes.c_int
        L.oracle_batch_dp.argtypes = [P, P, i32, P, P, i64, i64, i64, i64, P, P, i32]
        L.oracle_batch_dp.restype = ctypes.c_int
        L.oracle_batch_ungapped.argtypes = [P, P, i32, P, P, i64, i64, i64, P, P, i32]
        L.oracle_batch_ungapped.restype = ctypes.c_int
        L.oracle_batch_closed_form.argtypes = [P, P, i32, P, P, i64, i64, i64, P, P, i32]
        L.oracle_batch_closed_form.restype = ctypes.c_int
        L.oracle_batch_banded.argtypes = [P, P, i32, P, P, i64, i64, i64, i64, i32, P, P, i32]
        L.oracle_batch_banded.restype = ctypes.c_int
        L.oracle_local_align.argtypes = [P, i32, P, i32, i64, i64, i64, P, P, P, P, P, P, i64, P]
        L.oracle_local_align.restype = ctypes.c_int
        _lib = L
    return _lib


def encode(reads: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
    """Injective symbol->byte encoding (equality is all the DP looks at)."""
    table: Dict[str, int] = {}
    if all(r.isascii() for r in reads):
        buf = np.frombuffer("".join(reads).encode("ascii"), dtype=np.uint8)
    else:
        codes: List[int] = []
        for r in reads:
            for ch in r:
                if ch not in table:
                    if len(table) >= 256:
                        raise ValueError("more than 256 distinct symbols")
                    table[ch] = len(table)
                codes.append(table[ch])
        buf = np.asarray(codes, dtype=np.uint8)
    offs = np.zeros(len(reads) + 1, dtype=np.int64)
    np.cumsum([len(r) for r in reads], out=offs[1:])
    return np.ascontiguousarray(buf), offs


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def batch_dp(reads: Sequence[str], a_idx, b_idx, match=10, mismatch=-1, indel=INT32_MIN,
             threads: int = 0, encoded=None) -> Tuple[np.ndarray, np.ndarray]:
    seqs, offs = encoded if encoded is not None else encode(reads)
    a = np.ascontiguousarray(a_idx, dtype=np.int32)
    b = np.ascontiguousarray(b_idx, dtype=np.int32)
    sc = np.zeros(a.shape[0], np.int32)
    en = np.zeros(a.shape[0], np.int32)
    if seqs.size == 0:
        seqs = np.zeros(1, np.uint8)
    rc = lib().oracle_batch_dp(_ptr(seqs), _ptr(offs), len(offs) - 1, _ptr(a), _ptr(b), a.shape[0],
                               match, mismatch, indel, _ptr(sc), _ptr(en), threads)
    if rc != 0:
        raise RuntimeError(f"oracle_batch_dp failed rc={rc}")
    return sc, en


def batch_ungapped(reads: Sequence[str], a_idx, b_idx, match=10, mismatch=-1,
                   threads: int = 0, encoded=None) -> Tuple[np.ndarray, np.ndarray]:
    seqs, offs = encoded if encoded is not None else encode(reads)
    a = np.ascontiguousarray(a_idx, dtype=np.int32)
    b = np.ascontiguousarray(b_idx, dtype=np.int32)
    sc = np.zeros(a.shape[0], np.int32)
    en = np.zeros(a.shape[0], np.int32)
    if seqs.size == 0:
        seqs = np.zeros(1, np.uint8)
    rc = lib().oracle_batch_ungapped(_ptr(seqs), _ptr(offs), len(offs) - 1, _ptr(a), _ptr(b),
                                     a.shape[0], match, mismatch, _ptr(sc), _ptr(en), threads)
    if rc != 0:
        raise RuntimeError(f"oracle_batch_ungapped failed rc={rc}")
    return sc, en


def batch_closed_form(reads: Sequence[str], a_idx, b_idx, match=10, mismatch=-1,
                      threads: int = 0, encoded=None) -> Tuple[np.ndarray, np.ndarray]:
    """The optimised CPU closed form (64 bases per popcount; ACGT reads <= 256 bases): bench.py's
    second CPU-baseline line.  Equal to batch_ungapped, which tests check."""
    seqs, offs = encoded if encoded is not None else encode(reads)
    a = np.ascontiguousarray(a_idx, dtype=np.int32)
    b = np.ascontiguousarray(b_idx, dtype=np.int32)
    sc = np.zeros(a.shape[0], np.int32)
    en = np.zeros(a.shape[0], np.int32)
    if seqs.size == 0:
        seqs = np.zeros(1, np.uint8)
    rc = lib().oracle_batch_closed_form(_ptr(seqs), _ptr(offs), len(offs) - 1, _ptr(a), _ptr(b),
                                        a.shape[0], match, mismatch, _ptr(sc), _ptr(en), threads)
    if rc != 0:
        raise RuntimeError(f"oracle_batch_closed_form failed rc={rc}")
    return sc, en


def batch_banded(reads: Sequence[str], a_idx, b_idx, match=10, mismatch=-1, indel=-2, band=8,
                 threads: int = 0, encoded=None) -> Tuple[np.ndarray, np.ndarray]:
    """The build's banded seed-and-extend knob (oracle_overlap_banded; not a reference mode)."""
    seqs, offs = encoded if encoded is not None else encode(reads)
    a = np.ascontiguousarray(a_idx, dtype=np.int32)
    b = np.ascontiguousarray(b_idx, dtype=np.int32)
    sc = np.zeros(a.shape[0], np.int32)
    en = np.zeros(a.shape[0], np.int32)
    if seqs.size == 0:
        seqs = np.zeros(1, np.uint8)
    rc = lib().oracle_batch_banded(_ptr(seqs), _ptr(offs), len(offs) - 1, _ptr(a), _ptr(b), a.shape[0],
                                   match, mismatch, indel, band, _ptr(sc), _ptr(en), threads)
    if rc != 0:
        raise RuntimeError(f"oracle_batch_banded failed rc={rc}")
    return sc, en


def banded_py(s: str, t: str, match: int = 10, mismatch: int = -1, indel: int = -2,
              band: int = 8) -> Tuple[int, int]:
    """Pure-Python statement of the banded knob (small cases; cross-checks the C version).

    Seed j* = ungapped first argmax, d* = n - j*; the aligners.py:33-48 recurrence
    on cells with |(i - j) - d*| <= band, out-of-band predecessors = -inf; last-row
    strict '>' first argmax over in-band cells.
    """
    n, m = len(s), len(t)
    _, jstar = ungapped(s, t, match, mismatch)
    d = n - jstar
    NEG = None
    dp = [[0] * (m + 1) for _ in range(n + 1)]
    inb = lambda i, j: abs((i - j) - d) <= band  # noqa: E731
    for i in range(1, n + 1):
        for j in range(1, m + 1):
            if not inb(i, j):
                dp[i][j] = NEG
                continue
            cand_d = dp[i - 1][j - 1] + (match if s[i - 1] == t[j - 1] else mismatch)
            up = dp[i - 1][j] + indel if inb(i - 1, j) else NEG
            left = dp[i][j - 1] + indel if inb(i, j - 1) else NEG
            if (up is NEG or cand_d >= up) and (left is NEG or cand_d >= left):
                dp[i][j] = cand_d
            elif up is not NEG and (left is NEG or up >= left):
                dp[i][j] = up
            else:
                dp[i][j] = left
    best, end = None, -1
    for j in range(m + 1):
        if inb(n, j) and (best is None or dp[n][j] > best):
            best, end = dp[n][j], j
    return int(best), end


def local_strings(query: str, reference: str, bi: int, bj: int, ops) -> Tuple[str, str, str, int, int]:
    """Rebuild aligners.py:133-160's strings from a walk: ops (1 diag, 2 up, 3 left) from (bi, bj)."""
    aq, ar = [], []
    i, j = bi, bj
    for c in ops:
        if c == 1:
            aq.append(query[i - 1]); ar.append(reference[j - 1]); i -= 1; j -= 1
        elif c == 2:
            aq.append(query[i - 1]); ar.append("-"); i -= 1
        else:
            aq.append("-"); ar.append(reference[j - 1]); j -= 1
    aligned_query = "".join(reversed(aq))
    aligned_reference = "".join(reversed(ar))
    to_print = (f"\nTarget:   {aligned_reference}\n          {'|' * len(aligned_reference)}\nQuery:    "
                f"{aligned_query}")
    return to_print, aligned_reference, aligned_query, i, j


def local_alignment(query: str, reference: str, match_score: int = 10, mismatch: int = -1,
                    indel: int = -1):
    """aligners.py:85-167 through the C restatement: the reference's 6-tuple."""
    buf, _ = encode([query, reference])
    n, m = len(query), len(reference)
    qb = np.ascontiguousarray(buf[:n]) if n else np.zeros(1, np.uint8)
    rb = np.ascontiguousarray(buf[n:]) if m else np.zeros(1, np.uint8)
    out = [np.zeros(1, np.int32) for _ in range(5)]
    cap = n + m + 1
    ops = np.zeros(cap, np.int8)
    k = np.zeros(1, np.int64)
    rc = lib().oracle_local_align(_ptr(qb), n, _ptr(rb), m, match_score, mismatch, indel,
                                  *[_ptr(o) for o in out], _ptr(ops), cap, _ptr(k))
    if rc != 0:
        raise RuntimeError("oracle_local_align failed")
    score, bi, bj = int(out[0][0]), int(out[1][0]), int(out[2][0])
    to_print, a_r, a_q, _, start = local_strings(query, reference, bi, bj, ops[: int(k[0])].tolist())
    assert start == int(out[4][0])
    return to_print, a_r, a_q, score, start, bj


def align_read_or_contig_to_reference(read_or_contig: str, reference_genome: str, read_length: int,
                                      match_score: int = 10, mismatch: int = -1, indel: int = -1):
    """aligners.py:170-202: a shorter item is aligned to the reference's tail only."""
    L = len(read_or_contig)
    if L < read_length:
        tp, a_r, a_q, sc, st, en = local_alignment(read_or_contig, reference_genome[-L:],
                                                   match_score, mismatch, indel)
        return tp, a_r, a_q, sc, len(reference_genome) - L + st, len(reference_genome) - L + en
    return local_alignment(read_or_contig, reference_genome, match_score, mismatch, indel)


def dp_one(s: str, t: str, match=10, mismatch=-1, indel=INT32_MIN, want_tb=False):
    """Single pair through the C restatement; optionally returns the traceback table."""
    (buf, offs) = encode([s, t])
    n, m = len(s), len(t)
    sc = np.zeros(1, np.int32)
    en = np.zeros(1, np.int32)
    tb = np.zeros((n + 1) * (m + 1), np.int8) if want_tb else None
    sp = buf[: n] if n else np.zeros(1, np.uint8)
    tp = buf[n:] if m else np.zeros(1, np.uint8)
    sp = np.ascontiguousarray(sp); tp = np.ascontiguousarray(tp)
    rc = lib().oracle_overlap_dp(_ptr(sp), n, _ptr(tp), m, match, mismatch, indel, _ptr(sc), _ptr(en),
                                 _ptr(tb) if tb is not None else None)
    if rc != 0:
        raise RuntimeError("oracle_overlap_dp failed")
    if want_tb:
        return int(sc[0]), int(en[0]), tb.reshape(n + 1, m + 1)
    return int(sc[0]), int(en[0])


# ----------------------------------------------------------------------------- graph

def graph_nx_k(reads: Sequence[str], k: int = 5,
               scorer: Optional[Callable[[str, str], Tuple[int, int]]] = None):
    """Restatement of overlapGraphs.py:5-61 (returns DiGraph, read_copies)."""
    import networkx as nx
    assert k >= 0, "k-mer length must be non-negative"
    if scorer is None:
        scorer = lambda s, t: dp_one(s, t)
    copies: Dict[str, int] = {}
    for r in reads:
        copies[r] = copies.get(r, 0) + 1
    G = nx.DiGraph()
    for r, c in copies.items():
        for i in range(c):
            G.add_node(f"{r}_{i}")
    index: Dict[str, list] = {}
    if k > 0:
        for r, c in copies.items():
            key = r[:k] if len(r) >= k else r
            index.setdefault(key, []).append((r, c))
    for ra, ca in copies.items():
        key = ra[-k:] if len(ra) >= k > 0 else ra
        cands = index.get(key, []) if k > 0 else list(copies.items())
        for rb, cb in cands:
            if ra != rb:
                sc, en = scorer(ra, rb)
                for x in range(ca):
                    for y in range(cb):
                        G.add_edge(f"{ra}_{x}", f"{rb}_{y}", weight=sc, end_position=en)
    return G, copies


def remove_cycles(G):
    """Restatement of overlapGraphs.py:106-130 (remove_cycles_from_graph), the reference loop itself:
    networkx's find_cycle (orientation 'original'), then the cycle's first minimum-'weight' edge is
    removed, until no cycle is left.  In place; returns G.  Quadratic: small graphs only."""
    import networkx as nx
    while True:
        try:
            cycle = nx.find_cycle(G, orientation="original")
        except nx.NetworkXNoCycle:
            break
        u, v, _ = min(((u, v, G[u][v]["weight"]) for u, v, _ in cycle), key=lambda x: x[2])
        G.remove_edge(u, v)
    return G

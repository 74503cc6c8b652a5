"""Drop-ins for the reference's ``aligners.overlap_alignment`` (aligners.py:6-82),
``local_alignment`` (aligners.py:85-167) and ``align_read_or_contig_to_reference``
(aligners.py:170-202).

Same signature, defaults and 5-tuple return value:
``(alignment_to_print, align_s, align_t, best_score, alignment_end_position)``.
The DP fill and last-row argmax (aligners.py:27-57) run on the GPU:

* in the reference's regime (gaps cannot win, e.g. the default indel of
  -2**31) the ungapped kernel returns (score, end) and the backtrack of
  aligners.py:59-76 is all-diagonal, so ``align_s = s[n-L:]`` and
  ``align_t = t[end-L:end]`` with ``L = min(n, end)``;
* otherwise the DP kernel also returns the int8 traceback table of
  aligners.py:30,42-48 and the backtrack walks it on the host.

One call launches GPU work for a single pair; batch callers should use
``ovlgraph.engine.OverlapEngine.score`` (as ``overlapGraphs`` does).
"""
from __future__ import annotations

import threading
from typing import Tuple

from .engine import INDEL_DEFAULT, OverlapEngine, default_engine

_lock = threading.Lock()


def _format(align_s: str, align_t: str) -> str:
    # aligners.py:78
    return f"\nTarget:   {align_t}\n          {'|' * len(align_t)}\nQuery:    {align_s}"


def _walk(tb, s: str, t: str, n: int, end: int) -> Tuple[str, str]:
    """Backtrack of aligners.py:59-76 over the GPU-produced traceback table."""
    out_s, out_t = [], []
    i, j = n, end
    while i > 0 and j > 0:
        d = tb[i, j]
        if d == 0:
            out_s.append(s[i - 1]); out_t.append(t[j - 1]); i -= 1; j -= 1
        elif d == 1:
            out_s.append(s[i - 1]); out_t.append("-"); i -= 1
        else:
            out_s.append("-"); out_t.append(t[j - 1]); j -= 1
    return "".join(reversed(out_s)), "".join(reversed(out_t))


def overlap_alignment(s, t, match_score=10, mismatch=-1, indel=INDEL_DEFAULT, engine: OverlapEngine = None):
    """Best overlap of a suffix of ``s`` with ``t`` (overhangs free), as aligners.py:6-82."""
    n, m = len(s), len(t)
    eng = engine or default_engine()
    with _lock:
        eng.set_reads([s, t])
        kind = eng.plan(int(match_score), int(mismatch), int(indel))
        if kind == "ungapped":
            sc, en = eng.score([0], [1], int(match_score), int(mismatch), int(indel))
            score, end = int(sc[0]), int(en[0])
            L = min(n, end)
            align_s, align_t = s[n - L:], t[end - L:end]
        else:
            score, end, tb = eng.align_one(0, 1, n, m, int(match_score), int(mismatch), int(indel),
                                           traceback=True)
            align_s, align_t = _walk(tb, s, t, n, end)
    return _format(align_s, align_t), align_s, align_t, int(score), int(end)


def _local_strings(query: str, reference: str, bi: int, bj: int, ops) -> Tuple[str, str]:
    """aligners.py:133-153: rebuild the aligned strings from the walk (1 diag, 2 up, 3 left)."""
    aq, ar = [], []
    i, j = bi, bj
    for c in ops:
        if c == 1:
            aq.append(query[i - 1]); ar.append(reference[j - 1]); i -= 1; j -= 1
        elif c == 2:
            aq.append(query[i - 1]); ar.append("-"); i -= 1
        else:
            aq.append("-"); ar.append(reference[j - 1]); j -= 1
    return "".join(reversed(ar)), "".join(reversed(aq))


def local_alignment(query, reference, match_score=10, mismatch=-1, indel=-1, engine: OverlapEngine = None):
    """Best local alignment (aligners.py:85-167) on the GPU: the reference's 6-tuple
    ``(alignment_to_print, aligned_reference, aligned_query, best_score, start_pos, end_pos)``."""
    eng = engine or default_engine()
    with _lock:
        score, bi, bj, si, sj, ops = eng.local_align(query, reference, int(match_score), int(mismatch), int(indel))
    aligned_reference, aligned_query = _local_strings(query, reference, bi, bj, ops.tolist())
    # aligners.py:159-160
    to_print = (f"\nTarget:   {aligned_reference}\n          {'|' * len(aligned_reference)}\nQuery:    "
                f"{aligned_query}")
    return to_print, aligned_reference, aligned_query, score, sj, bj


def align_read_or_contig_to_reference(read_or_contig, reference_genome, read_length, match_score=10, mismatch=-1,
                                      indel=-1, engine: OverlapEngine = None):
    """aligners.py:170-202: an item shorter than ``read_length`` is aligned to the reference's
    tail of the same length and its positions shifted back; otherwise to the whole reference."""
    L = len(read_or_contig)
    if L < read_length:
        tail = reference_genome[-L:]  # as aligners.py:189 (L = 0: the whole reference)
        tp, a_r, a_q, sc, st, en = local_alignment(read_or_contig, tail, match_score, mismatch, indel, engine)
        return tp, a_r, a_q, sc, len(reference_genome) - L + st, len(reference_genome) - L + en
    return local_alignment(read_or_contig, reference_genome, match_score, mismatch, indel, engine)

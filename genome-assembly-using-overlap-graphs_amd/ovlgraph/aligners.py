"""Drop-in for the reference's ``aligners.overlap_alignment`` (aligners.py:6-82).

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

"""Drop-in graph builders of the reference's ``overlapGraphs.py``, scored on the GPU.

``construct_overlap_graph_nx_k(reads, k=5)`` (overlapGraphs.py:5-61) returns the
same ``(nx.DiGraph, read_copies)``: node names ``f"{read}_{copy}"`` inserted in
``read_copies`` order (:22-28), edges inserted per candidate pair in the
reference's enumeration order and then per (copy_a, copy_b) (:43-60), with the
attributes ``weight`` (score) and ``end_position`` as Python ints.  The only
change is *how* the list is built and scored: the k-mer candidate list is
enumerated on the GPU (``OverlapEngine.candidates``; the host restatement
``candidates.enumerate_candidates`` when asked, or when the keys do not fit the
device's 64-bit keys) and scored in one batched GPU call instead of one
``overlap_alignment`` call per pair (:53).

Also provided: ``construct_overlap_graph_string`` (:196-232) and
``construct_string_graph`` (:332-351), which score all ordered pairs / all
``combinations`` and keep edges with ``score > 0``; and ``build_overlap_graph``,
the name BASELINE.json's north_star uses, as an alias.

Layout, cycle removal and contig walking (:64-193) consume this graph and are
out of scope.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import networkx as nx
import numpy as np

from ._lib import OvlError
from .candidates import dedup_reads, enumerate_candidates
from .engine import INDEL_DEFAULT, OverlapEngine, default_engine

CANDIDATE_MODES = ("auto", "device", "host")


def _score(distinct: Sequence[str], a: np.ndarray, b: np.ndarray, engine: Optional[OverlapEngine],
           scorer=None) -> Tuple[List[int], List[int]]:
    if a.shape[0] == 0:
        return [], []
    if scorer is not None:  # (score, end) arrays from another backend, e.g. the sharded path
        sc, en = scorer(distinct, a, b)
    else:
        eng = engine or default_engine()
        eng.set_reads(distinct)
        sc, en = eng.score(a, b, 10, -1, INDEL_DEFAULT)
    return np.asarray(sc).tolist(), np.asarray(en).tolist()


def _node_names(distinct: Sequence[str], counts: Sequence[int]) -> List[List[str]]:
    return [[f"{r}_{c}" for c in range(cnt)] for r, cnt in zip(distinct, counts)]


def assemble_graph(distinct: Sequence[str], counts: Sequence[int], a, b, score, end,
                   min_score: Optional[int] = None) -> nx.DiGraph:
    """Build the DiGraph from scored candidates in reference insertion order.

    Nodes: every copy of every distinct read (overlapGraphs.py:25-28).
    Edges: for each pair p in order, for each copy of a, for each copy of b
    (overlapGraphs.py:55-60); with ``min_score`` set, pairs scoring
    ``<= min_score`` are dropped (overlapGraphs.py:225).
    """
    names = _node_names(distinct, counts)
    G = nx.DiGraph()
    G.add_nodes_from(n for group in names for n in group)
    a_l = a.tolist() if hasattr(a, "tolist") else list(a)
    b_l = b.tolist() if hasattr(b, "tolist") else list(b)
    s_l = score.tolist() if hasattr(score, "tolist") else list(score)
    e_l = end.tolist() if hasattr(end, "tolist") else list(end)

    def edges():
        for ia, ib, sc, en in zip(a_l, b_l, s_l, e_l):
            if min_score is not None and sc <= min_score:
                continue
            for u in names[ia]:
                for v in names[ib]:
                    yield u, v, {"weight": sc, "end_position": en}

    G.add_edges_from(edges())
    return G


def candidates_and_scores(distinct: Sequence[str], k: int, engine: Optional[OverlapEngine] = None, scorer=None,
                          candidates: str = "auto"):
    """Candidate pairs (overlapGraphs.py:30-52) and their (score, end) (:53), in reference order.

    ``candidates``: "device" enumerates on the GPU (list kept resident and scored
    without a host round trip), "host" uses ``enumerate_candidates``, "auto" is
    "device" unless the k-mer keys do not fit the device path (OVL_E_UNSUPPORTED).
    A custom ``scorer`` (e.g. the sharded path) always gets host-enumerated pairs.
    """
    if candidates not in CANDIDATE_MODES:
        raise ValueError(f"candidates must be one of {CANDIDATE_MODES}")
    if scorer is not None or candidates == "host":
        a, b = enumerate_candidates(distinct, k)
        sc, en = _score(distinct, a, b, engine, scorer)
        return a, b, sc, en
    eng = engine or default_engine()
    eng.set_reads(distinct)
    try:
        a, b = eng.candidates(k)
    except OvlError as e:
        if e.code != -4 or candidates == "device":
            raise
        a, b = enumerate_candidates(distinct, k)
        sc, en = _score(distinct, a, b, eng, None)
        return a, b, sc, en
    sc, en = eng.score_candidates(10, -1, INDEL_DEFAULT)
    return a, b, sc.tolist(), en.tolist()


def construct_overlap_graph_nx_k(reads, k=5, engine: Optional[OverlapEngine] = None, scorer=None,
                                 candidates: str = "auto"):
    """Overlap graph over k-mer-filtered candidates (overlapGraphs.py:5-61)."""
    assert k >= 0, "k-mer length must be non-negative"
    distinct, counts = dedup_reads(reads)
    a, b, sc, en = candidates_and_scores(distinct, k, engine, scorer, candidates)
    G = assemble_graph(distinct, counts, a, b, sc, en)
    return G, dict(zip(distinct, counts))


build_overlap_graph = construct_overlap_graph_nx_k


def construct_overlap_graph_string(reads, engine: Optional[OverlapEngine] = None, scorer=None,
                                   candidates: str = "auto"):
    """All ordered distinct pairs, edges where score > 0 (overlapGraphs.py:196-232)."""
    distinct, counts = dedup_reads(reads)
    a, b, sc, en = candidates_and_scores(distinct, 0, engine, scorer, candidates)
    G = assemble_graph(distinct, counts, a, b, sc, en, min_score=0)
    return G, dict(zip(distinct, counts))


def construct_string_graph(reads, engine: Optional[OverlapEngine] = None, scorer=None):
    """Raw reads as nodes, ``combinations(reads, 2)`` scored, edges where score > 0 (:332-351)."""
    reads = list(reads)
    G = nx.DiGraph()
    G.add_nodes_from(reads)
    distinct, _ = dedup_reads(reads)
    index: Dict[str, int] = {r: i for i, r in enumerate(distinct)}
    ids = np.fromiter((index[r] for r in reads), dtype=np.int32, count=len(reads))
    n = len(reads)
    if n >= 2:
        iu, ju = np.triu_indices(n, k=1)  # combinations order: i-major, j ascending
        a, b = ids[iu], ids[ju]
    else:
        a = b = np.zeros(0, dtype=np.int32)
    sc, en = _score(distinct, np.ascontiguousarray(a), np.ascontiguousarray(b), engine, scorer)
    G.add_edges_from((distinct[x], distinct[y], {"weight": s, "end_position": e})
                     for x, y, s, e in zip(a.tolist(), b.tolist(), sc, en) if s > 0)
    print(f"graph: {G.edges}")
    return G

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

``remove_cycles_from_graph`` (:106-130) removes the same edges as the
reference's find_cycle / remove-weakest-edge loop, through an exact replay of
that loop in native code (``ovl_remove_cycles``) that does not restart its DFS
after each removal.  Topological sorting and contig walking (:64-103, :133-193)
stay networkx/Python.
"""
from __future__ import annotations

import gc
import os
from typing import Dict, List, Optional, Sequence, Tuple

import networkx as nx
import numpy as np

from ._lib import OvlError
from .candidates import dedup_reads, enumerate_candidates
from .engine import INDEL_DEFAULT, OverlapEngine, default_engine

CANDIDATE_MODES = ("auto", "device", "host")


def _score(distinct: Sequence[str], a: np.ndarray, b: np.ndarray, engine: Optional[OverlapEngine],
           scorer=None, encoded=None) -> Tuple[np.ndarray, np.ndarray]:
    """(score, end) int32 arrays of the pairs (a, b) in one batched call (or through ``scorer``)."""
    if a.shape[0] == 0:
        return np.zeros(0, np.int32), np.zeros(0, np.int32)
    if scorer is not None:  # (score, end) arrays from another backend, e.g. the sharded path
        sc, en = scorer(distinct, a, b)
    else:
        eng = engine or default_engine()
        eng.set_reads(distinct, encoded)
        sc, en = eng.score(a, b, 10, -1, INDEL_DEFAULT)
    return np.asarray(sc, dtype=np.int32), np.asarray(en, dtype=np.int32)


class _Stages:
    """Wall-clock stages of a graph build into a caller's dict (``timing=``), or nothing."""

    def __init__(self, out: Optional[dict]):
        import time
        self.out, self._clock = out, time.perf_counter
        self._t = self._clock()

    def __call__(self, name: str) -> None:
        if self.out is not None:
            t = self._clock()
            self.out[name] = self.out.get(name, 0.0) + (t - self._t)
            self._t = t


def _node_names(distinct: Sequence[str], counts: Sequence[int]) -> List[List[str]]:
    return [[f"{r}_{c}" for c in range(cnt)] for r, cnt in zip(distinct, counts)]


def assemble_graph(distinct: Sequence[str], counts: Sequence[int], a, b, score, end,
                   min_score: Optional[int] = None) -> nx.DiGraph:
    """Build the DiGraph from scored candidates in reference insertion order, through
    networkx's own ``add_edges_from`` (the plain statement; ``assemble_graph_direct``
    builds the identical graph faster and is what the builders use).

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
                          candidates: str = "auto", timing: Optional[dict] = None):
    """Candidate pairs (overlapGraphs.py:30-52) and their (score, end) (:53), in reference order, as
    int32 arrays.

    ``candidates``: "device" enumerates on the GPU (list kept resident and scored
    without a host round trip), "host" uses ``enumerate_candidates``, "auto" is
    "device" unless the k-mer keys do not fit the device path (OVL_E_UNSUPPORTED).
    A custom ``scorer`` (e.g. the sharded path) always gets host-enumerated pairs.
    ``timing``: a dict that receives the stage times (s): encode, set_reads, enumerate,
    candidates_copy, score (host enumeration: enumerate_host).
    """
    from .engine import encode_reads
    if candidates not in CANDIDATE_MODES:
        raise ValueError(f"candidates must be one of {CANDIDATE_MODES}")
    st = _Stages(timing)
    if scorer is not None or candidates == "host":
        a, b = enumerate_candidates(distinct, k)
        st("enumerate_host")
        sc, en = _score(distinct, a, b, engine, scorer)
        st("score")
        return a, b, sc, en
    eng = engine or default_engine()
    enc = encode_reads(distinct)
    st("encode")
    eng.set_reads(distinct, enc)
    st("set_reads")
    try:
        n = eng.enumerate_candidates(k)
    except OvlError as e:
        if e.code != -4 or candidates == "device":
            raise
        a, b = enumerate_candidates(distinct, k)
        st("enumerate_host")
        sc, en = _score(distinct, a, b, eng, None, enc)
        st("score")
        return a, b, sc, en
    st("enumerate")
    a, b = eng.candidates_copy(n)
    st("candidates_copy")
    sc, en = eng.score_candidates(10, -1, INDEL_DEFAULT)
    st("score")
    return a, b, sc, en


def assemble_graph_direct(distinct: Sequence[str], counts: Sequence[int], a, b, score, end,
                          min_score: Optional[int] = None, native: Optional[bool] = None) -> nx.DiGraph:
    """``assemble_graph`` without networkx's per-edge ``add_edge`` overhead.

    Builds the DiGraph's own node / successor / predecessor dicts in bulk, in the
    reference's insertion order (overlapGraphs.py:25-28 nodes; :55-60 edges per pair,
    per copy of a, per copy of b), with one attribute dict per edge shared by its
    successor and predecessor entries -- the structure ``add_edge`` builds, so every
    networkx view (edges, successors, predecessors, data) reads identically:

    * pairs x copies are expanded into edge arrays (u, v node ids) with numpy;
    * successor dicts: edges stably sorted by u keep the global order per u;
    * predecessor dicts: edges stably sorted by v keep the global order per v.

    The dicts are built by the C extension (csrc/ovl_digraph.c) in one pass over the edges when it is
    built (``native=None``: when available; True: required; False: the Python grouping below).
    """
    # millions of new dicts: the cyclic GC would re-traverse them at every generation-2 pass
    # (they hold no cycles), so it is paused for the bulk build
    gc_was = gc.isenabled()
    gc.disable()
    try:
        return _assemble_direct(distinct, counts, a, b, score, end, min_score, native)
    finally:
        if gc_was:
            gc.enable()


_digraph_mod = None


def _digraph():
    """The C builder of the adjacency dicts (build/_digraph*.so, csrc/ovl_digraph.c), or None if not built."""
    global _digraph_mod
    if _digraph_mod is None:
        import importlib.machinery
        import importlib.util
        import os
        import sysconfig
        from ._lib import PKG_ROOT
        path = os.path.join(PKG_ROOT, "build", "_digraph" + sysconfig.get_config_var("EXT_SUFFIX"))
        _digraph_mod = False
        if os.path.exists(path):
            spec = importlib.util.spec_from_file_location("ovlgraph._digraph", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            # (its builder calls take the graph's dicts from pooled, huge-page-advised object arenas while they run:
            # csrc/ovl_digraph.c arena_pool; OVL_ARENA_POOL=0 leaves CPython's allocator)
            _digraph_mod = mod
    return _digraph_mod or None


class _EdgeAttrs:
    """Its instances' ``__dict__`` is a key-sharing dict (PEP 412) with the two edge attributes; the C builder
    copies it, so every edge's attribute dict shares one key table (values only per edge)."""


def _attr_template() -> dict:
    t = _EdgeAttrs()
    t.weight = None
    t.end_position = None
    return t.__dict__


def _assemble_direct(distinct, counts, a, b, score, end, min_score, native: Optional[bool] = None):
    names = _node_names(distinct, counts)
    order = [n for group in names for n in group]
    cnt = np.fromiter((len(g) for g in names), dtype=np.int64, count=len(names))
    first = np.zeros(len(names) + 1, dtype=np.int64)
    np.cumsum(cnt, out=first[1:])
    a_arr = np.asarray(a, dtype=np.int64)
    b_arr = np.asarray(b, dtype=np.int64)
    s_arr = np.asarray(score)
    e_arr = np.asarray(end)
    if min_score is not None and a_arr.shape[0]:
        keep = s_arr > min_score
        a_arr, b_arr, s_arr, e_arr = a_arr[keep], b_arr[keep], s_arr[keep], e_arr[keep]
    # edges of pair p: k = 0 .. ca*cb-1 -> (copy of a = k // cb, copy of b = k % cb)
    per = cnt[a_arr] * cnt[b_arr]
    n_e = int(per.sum())
    pid = np.repeat(np.arange(a_arr.shape[0], dtype=np.int64), per)
    start = np.zeros(a_arr.shape[0], dtype=np.int64)
    if a_arr.shape[0]:
        np.cumsum(per[:-1], out=start[1:])
    k = np.arange(n_e, dtype=np.int64) - start[pid]
    cb = cnt[b_arr][pid]
    u = first[a_arr][pid] + k // cb
    v = first[b_arr][pid] + k % cb
    mod = _digraph() if native is not False else None
    if native and mod is None:
        raise RuntimeError("ovlgraph._digraph is not built (make -C genome-assembly-using-overlap-graphs_amd/csrc)")
    if mod is not None:
        # one pass in C over the edges in insertion order: the same dicts as the grouped build below
        G = nx.DiGraph()
        node, succ, pred = mod.build(order, np.ascontiguousarray(u, np.int64), np.ascontiguousarray(v, np.int64),
                                     np.ascontiguousarray(s_arr[pid], np.int32),
                                     np.ascontiguousarray(e_arr[pid], np.int32), _attr_template())
        G._node = node
        G._succ = succ
        G._pred = pred
        nx._clear_cache(G)
        return G
    dicts = [{"weight": sc, "end_position": en}
             for sc, en in zip(s_arr[pid].tolist(), e_arr[pid].tolist())]
    n_nodes = len(order)

    def grouped(key, other):
        # per node (in node order) the dict other-name -> edge dict, edges in global order
        perm = np.argsort(key, kind="stable")
        bounds = np.searchsorted(key[perm], np.arange(n_nodes + 1, dtype=np.int64))
        names_sorted = [order[x] for x in other[perm].tolist()]
        dicts_sorted = [dicts[x] for x in perm.tolist()]
        bl = bounds.tolist()
        return {order[n]: dict(zip(names_sorted[bl[n]:bl[n + 1]], dicts_sorted[bl[n]:bl[n + 1]]))
                for n in range(n_nodes)}

    G = nx.DiGraph()
    G._node = {n: {} for n in order}
    G._succ = grouped(u, v)   # descriptor: sets _adj and _succ, resets cached views
    G._pred = grouped(v, u)
    nx._clear_cache(G)
    return G


class OverlapEdges:
    """Columnar overlap edges: the scored candidate list before networkx.

    ``reads`` / ``counts`` are ``read_copies`` (overlapGraphs.py:18-20) as two lists;
    ``a``, ``b``, ``score``, ``end`` are int32 arrays in the reference's pair order
    (overlapGraphs.py:43-53).  Every pair stands for ``counts[a] * counts[b]`` edges
    (one per copy pair, :55-60).  ``to_digraph()`` gives the reference's DiGraph: lazy (its dicts
    are built on first use) unless ``lazy=False``.
    """

    def __init__(self, reads, counts, a, b, score, end, min_score: Optional[int] = None):
        self.reads = list(reads)
        self.counts = list(counts)
        self.a = np.ascontiguousarray(a, dtype=np.int32)
        self.b = np.ascontiguousarray(b, dtype=np.int32)
        self.score = np.ascontiguousarray(score, dtype=np.int32)
        self.end = np.ascontiguousarray(end, dtype=np.int32)
        self.min_score = min_score  # edges kept only when score > min_score (overlapGraphs.py:225)

    def __len__(self) -> int:
        return int(self.a.shape[0])

    def read_copies(self) -> Dict[str, int]:
        return dict(zip(self.reads, self.counts))

    def node_names(self) -> List[str]:
        return [n for group in _node_names(self.reads, self.counts) for n in group]

    def kept(self) -> np.ndarray:
        return np.ones(len(self), bool) if self.min_score is None else self.score > self.min_score

    def n_nodes(self) -> int:
        return int(sum(self.counts))

    def n_edges(self) -> int:
        c = np.asarray(self.counts, dtype=np.int64)
        k = self.kept()
        return int((c[self.a[k]] * c[self.b[k]]).sum()) if len(self) else 0

    def edge_arrays(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """(u, v, weight, end_position) per edge, u/v indexing ``node_names()``, in insertion order."""
        c = np.asarray(self.counts, dtype=np.int64)
        first = np.zeros(c.shape[0] + 1, dtype=np.int64)
        np.cumsum(c, out=first[1:])
        k = self.kept()
        a, b = self.a[k].astype(np.int64), self.b[k].astype(np.int64)
        per = c[a] * c[b]
        pid = np.repeat(np.arange(a.shape[0], dtype=np.int64), per)
        start = np.zeros(a.shape[0], dtype=np.int64)
        if a.shape[0]:
            np.cumsum(per[:-1], out=start[1:])
        q = np.arange(pid.shape[0], dtype=np.int64) - start[pid]
        cb = c[b][pid]
        return (first[a][pid] + q // cb, first[b][pid] + q % cb, self.score[k][pid], self.end[k][pid])

    def _keep_mask(self):
        return None if self.min_score is None else np.ascontiguousarray(self.kept(), dtype=np.uint8)

    def csr(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """The graph's successor lists as CSR (off int64, heads int32, weights int64) in node order and, per
        node, insertion order -- what ``remove_cycles_from_graph`` replays -- straight from the columns."""
        mod = _digraph()
        if mod is None:
            raise RuntimeError("ovlgraph._digraph is not built (make -C genome-assembly-using-overlap-graphs_amd/csrc)")
        boff, bh, bw = mod.overlap_csr(np.ascontiguousarray(self.counts, dtype=np.int32), self.a, self.b, self.score,
                                       self._keep_mask())
        off = np.frombuffer(boff, dtype=np.int64)
        n = int(off[-1])
        return off, np.frombuffer(bh, dtype=np.int32, count=n), np.frombuffer(bw, dtype=np.int64, count=n)

    def _dicts(self, alive: Optional[np.ndarray] = None):
        """(node, succ, pred) dicts of the DiGraph, for the edges whose CSR index (``csr()``) is alive."""
        mod = _digraph()
        gc_was = gc.isenabled()
        gc.disable()  # millions of new dicts with no cycles: no collector passes over them while they are built
        try:
            if mod is not None:
                return mod.build_overlap(self.node_names(), np.ascontiguousarray(self.counts, dtype=np.int32),
                                         self.a, self.b, self.score, self.end, self._keep_mask(),
                                         None if alive is None else np.ascontiguousarray(alive, dtype=np.uint8),
                                         _attr_template())
            if alive is not None:
                raise RuntimeError("ovlgraph._digraph is not built: no survivors-only build")
            G = _assemble_direct(self.reads, self.counts, self.a, self.b, self.score, self.end, self.min_score,
                                 False)
            return G._node, G._succ, G._pred
        finally:
            if gc_was:
                gc.enable()

    def to_digraph(self, lazy: bool = True) -> nx.DiGraph:
        """The reference's DiGraph (overlapGraphs.py:22-60): a ``LazyOverlapDiGraph`` over these columns, or
        with ``lazy=False`` one whose dicts are built now."""
        if lazy and _digraph() is not None:
            return LazyOverlapDiGraph._over(self)
        return assemble_graph_direct(self.reads, self.counts, self.a, self.b, self.score, self.end,
                                     self.min_score)


class _Materialise:
    """Data descriptor for a DiGraph dict attribute of ``LazyOverlapDiGraph``: the first read builds the
    dicts from the columns (and the object becomes a plain ``nx.DiGraph``); a write (networkx's own
    ``__init__``, or a caller replacing the dicts) makes it a plain DiGraph first."""

    def __init__(self, name: str):
        self.name = name

    def __get__(self, obj, owner=None):
        if obj is None:
            return self
        obj._materialise()
        return obj.__dict__[self.name]

    def __set__(self, obj, value):
        if "_ovl_edges" in obj.__dict__:
            obj._materialise()
        obj.__class__ = nx.DiGraph
        setattr(obj, self.name, value)


class LazyOverlapDiGraph(nx.DiGraph):
    """The overlap graph of ``construct_overlap_graph_nx_k`` before its dicts exist.

    It is an ``nx.DiGraph`` over the columns of ``OverlapEdges``: the node / successor / predecessor dicts
    (the structure ``add_edge`` builds, overlapGraphs.py:22-60) are built in C on the first access to any
    of them, after which the object *is* a plain ``nx.DiGraph`` (its class is switched), so every view,
    mutation and networkx algorithm behaves as on the reference's graph.  Until then node and edge counts
    come from the columns, and ``remove_cycles_from_graph`` replays the cycle removal on a CSR built from
    the columns and materialises only the surviving edges.
    """

    _node = _Materialise("_node")
    _adj = _Materialise("_adj")
    _succ = _adj
    _pred = _Materialise("_pred")

    @classmethod
    def _over(cls, edges: "OverlapEdges") -> "LazyOverlapDiGraph":
        G = cls.__new__(cls)
        od = G.__dict__
        od["graph"] = {}
        od["__networkx_cache__"] = {}
        od["_ovl_edges"] = edges
        return G

    def _materialise(self, alive: Optional[np.ndarray] = None) -> None:
        od = self.__dict__
        edges = od.get("_ovl_edges")
        if edges is None:
            return
        self._install(*edges._dicts(alive))

    def _install(self, node, succ, pred) -> None:
        """Become the plain ``nx.DiGraph`` with these dicts."""
        od = self.__dict__
        od.pop("_ovl_edges", None)
        self.__class__ = nx.DiGraph
        self._node = node
        self._succ = succ   # (networkx's descriptor: sets _adj and _succ, drops cached views)
        self._pred = pred
        nx._clear_cache(self)

    @property
    def is_materialised(self) -> bool:
        return "_ovl_edges" not in self.__dict__

    def __len__(self) -> int:
        e = self.__dict__.get("_ovl_edges")
        return e.n_nodes() if e is not None else super().__len__()

    def number_of_nodes(self) -> int:
        return len(self)

    def number_of_edges(self, u=None, v=None) -> int:
        e = self.__dict__.get("_ovl_edges")
        if e is not None and u is None and v is None:
            return e.n_edges()
        return super().number_of_edges(u, v)


_engines: Dict[Tuple[int, ...], OverlapEngine] = {}


def engine_on(devices) -> OverlapEngine:
    """A cached engine over ``devices`` ("all" or a list of ordinals): one process, several GPUs."""
    key = ("all",) if devices == "all" else tuple(int(d) for d in devices)
    if key not in _engines:
        _engines[key] = OverlapEngine(devices="all" if key == ("all",) else list(key))
    return _engines[key]


def overlap_edges_k(reads, k=5, engine: Optional[OverlapEngine] = None, scorer=None,
                    candidates: str = "auto", devices=None, timing: Optional[dict] = None) -> OverlapEdges:
    """Scored k-mer candidates of ``construct_overlap_graph_nx_k`` as columns (no networkx).
    ``timing``: a dict that receives the stage times (s), dedup first (candidates_and_scores)."""
    assert k >= 0, "k-mer length must be non-negative"
    if engine is None and devices is not None:
        engine = engine_on(devices)
    st = _Stages(timing)
    distinct, counts = dedup_reads(reads)
    st("dedup")
    a, b, sc, en = candidates_and_scores(distinct, k, engine, scorer, candidates, timing)
    return OverlapEdges(distinct, counts, a, b, sc, en)


def construct_overlap_graph_nx_k(reads, k=5, engine: Optional[OverlapEngine] = None, scorer=None,
                                 candidates: str = "auto", devices=None):
    """Overlap graph over k-mer-filtered candidates (overlapGraphs.py:5-61).

    ``devices`` ("all" or ordinals) scores on several GPUs from this one process: every
    device enumerates the same list, scores its Σ n·m-balanced shard and copies its
    results into its slice of the host result arrays."""
    edges = overlap_edges_k(reads, k, engine, scorer, candidates, devices)
    return edges.to_digraph(), edges.read_copies()


build_overlap_graph = construct_overlap_graph_nx_k


def construct_overlap_graph_string(reads, engine: Optional[OverlapEngine] = None, scorer=None,
                                   candidates: str = "auto"):
    """All ordered distinct pairs, edges where score > 0 (overlapGraphs.py:196-232)."""
    distinct, counts = dedup_reads(reads)
    a, b, sc, en = candidates_and_scores(distinct, 0, engine, scorer, candidates)
    edges = OverlapEdges(distinct, counts, a, b, sc, en, min_score=0)
    return edges.to_digraph(), edges.read_copies()


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
                     for x, y, s, e in zip(a.tolist(), b.tolist(), sc.tolist(), en.tolist()) if s > 0)
    print(f"graph: {G.edges}")
    return G


def _csr_python(nodes, adj):
    """The successor lists as CSR (node order, adjacency order within a node) -- Python passes."""
    index = {v: i for i, v in enumerate(nodes)}
    deg = np.fromiter((len(adj[u]) for u in nodes), dtype=np.int64, count=len(nodes))
    off = np.zeros(len(nodes) + 1, dtype=np.int64)
    np.cumsum(deg, out=off[1:])
    n_edges = int(off[-1])
    heads = np.fromiter((index[v] for u in nodes for v in adj[u]), dtype=np.int32, count=n_edges)
    wlist = [d["weight"] for u in nodes for d in adj[u].values()]
    if not all(isinstance(w, (int, np.integer)) and not isinstance(w, bool) for w in wlist):
        raise TypeError("remove_cycles_from_graph needs an integer 'weight' on every edge")
    weights = np.array(wlist, dtype=np.int64) if wlist else np.zeros(0, dtype=np.int64)
    return off, heads, weights


# the lazy path's replay and dict build overlapped (build_overlap_stream); OVL_CYCLES_STREAM=0 runs them one after
# the other (tests compare both)
_STREAM_OFF = os.environ.get("OVL_CYCLES_STREAM", "1") == "0"


def remove_cycles_from_graph(overlap_graph, native_edges: Optional[bool] = None, timing: Optional[dict] = None):
    """Remove the weakest edge of the first cycle networkx's ``find_cycle`` reports until the
    graph is a DAG (overlapGraphs.py:106-130), in place; returns the graph.

    Removes exactly the reference's edges (same cycles, same ``weight`` minimum, first in cycle
    order on ties), in the same order, by replaying its DFS in ``ovl_remove_cycles`` (C++,
    csrc/ovl_graph.cpp).  ``weight`` must be an integer on every edge.

    The per-edge passes around the replay -- the successor lists as CSR, and the removals
    (``del succ[u][v]; del pred[v][u]`` per edge, as ``DiGraph.remove_edge``, one cache clear at the
    end) -- run in the C extension (csrc/ovl_digraph.c) when it is built (``native_edges=None``;
    True: required; False: Python passes).  ``timing``: a dict that receives the stage times (s).
    """
    import ctypes
    import time
    from . import _lib
    G = overlap_graph
    t0 = time.perf_counter()
    mod = _digraph() if native_edges is not False else None
    if native_edges and mod is None:
        raise RuntimeError("ovlgraph._digraph is not built (make -C genome-assembly-using-overlap-graphs_amd/csrc)")
    if mod is not None and type(G) is LazyOverlapDiGraph and not G.is_materialised:
        # still columns: the replay's CSR straight from them, then the dicts of the surviving edges only -- built
        # while the replay runs (on a second thread, build_overlap_stream): a node's successors as soon as its
        # out-edges are final, the predecessors once the replay is done
        edges = G.__dict__["_ovl_edges"]
        off, heads, weights = edges.csr()
        t1 = time.perf_counter()
        if hasattr(mod, "build_overlap_stream") and not _STREAM_OFF:
            fn = ctypes.cast(_lib.load().ovl_remove_cycles_stream, ctypes.c_void_p).value
            gc_was = gc.isenabled()
            gc.disable()  # (as _dicts: millions of new dicts with no cycles)
            try:
                node, succ, pred, _rem, n_removed = mod.build_overlap_stream(
                    edges.node_names(), np.ascontiguousarray(edges.counts, dtype=np.int32), edges.a, edges.b,
                    edges.score, edges.end, edges._keep_mask(), _attr_template(), fn,
                    np.ascontiguousarray(off, dtype=np.int64), np.ascontiguousarray(heads, dtype=np.int32),
                    np.ascontiguousarray(weights, dtype=np.int64))
            finally:
                if gc_was:
                    gc.enable()
            G._install(node, succ, pred)
            t3 = time.perf_counter()
            if timing is not None:
                timing.update(csr=t1 - t0, replay=t3 - t1, remove=0.0, removed=int(n_removed), lazy=True,
                              overlapped=True)
            return G
        removed, n_removed = _replay(off, heads, weights)
        t2 = time.perf_counter()
        alive = np.ones(heads.shape[0], dtype=np.uint8)
        alive[removed[:n_removed]] = 0
        G._materialise(alive)
        t3 = time.perf_counter()
        if timing is not None:
            timing.update(csr=t1 - t0, replay=t2 - t1, remove=t3 - t2, removed=int(n_removed), lazy=True,
                          overlapped=False)
        return G
    nodes = list(G)
    adj = G._adj
    if native_edges and mod is None:
        raise RuntimeError("ovlgraph._digraph is not built (make -C genome-assembly-using-overlap-graphs_amd/csrc)")
    # the C passes need networkx's own DiGraph (plain dicts; remove_edge not overridden)
    got = mod.csr(nodes, adj, np.integer) if mod is not None and type(G) is nx.DiGraph and type(adj) is dict else None
    if got is not None:
        boff, bheads, bw = got
        off = np.frombuffer(boff, dtype=np.int64)
        n_edges = int(off[-1])
        heads = np.frombuffer(bheads, dtype=np.int32, count=n_edges)
        weights = np.frombuffer(bw, dtype=np.int64, count=n_edges)
    else:
        mod = None
        off, heads, weights = _csr_python(nodes, adj)
        n_edges = int(off[-1])
    t1 = time.perf_counter()
    removed, n_rem = _replay(off, heads, weights)
    t2 = time.perf_counter()
    if n_rem:
        # CSR index -> (u, v): the tail is the node whose adjacency range holds the index
        idx = removed[:n_rem]
        tails = np.searchsorted(off, idx, side="right") - 1
        if mod is not None:
            try:
                mod.remove_edges(G._succ, G._pred, nodes, np.ascontiguousarray(tails, np.int64),
                                 heads[idx].astype(np.int64))
            finally:
                nx._clear_cache(G)
        else:
            for t, e in zip(tails.tolist(), idx.tolist()):
                G.remove_edge(nodes[t], nodes[heads[e]])
    t3 = time.perf_counter()
    if timing is not None:
        timing.update(csr=t1 - t0, replay=t2 - t1, remove=t3 - t2, removed=int(n_rem), lazy=False)
    return G


def _replay(off: np.ndarray, heads: np.ndarray, weights: np.ndarray) -> Tuple[np.ndarray, int]:
    """ovl_remove_cycles over a CSR graph: (removed CSR indices in removal order, their count)."""
    import ctypes
    from . import _lib
    n_nodes = off.shape[0] - 1
    removed = np.zeros(max(heads.shape[0], 1), dtype=np.int64)
    n_removed = ctypes.c_int64(0)
    off = np.ascontiguousarray(off, dtype=np.int64)
    heads = np.ascontiguousarray(heads, dtype=np.int32)
    weights = np.ascontiguousarray(weights, dtype=np.int64)
    _lib.check(_lib.load().ovl_remove_cycles(off.ctypes.data_as(ctypes.c_void_p), heads.ctypes.data_as(ctypes.c_void_p),
                                             weights.ctypes.data_as(ctypes.c_void_p), n_nodes,
                                             removed.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n_removed)))
    return removed, int(n_removed.value)


def topological_sort(dag):
    """overlapGraphs.py:133-148: networkx's topological order, ValueError on a cycle."""
    print("Sorting graph topologically...")
    try:
        return list(nx.topological_sort(dag))
    except nx.NetworkXUnfeasible:
        raise ValueError("Graph is not a DAG! Cycles still exist.")


def create_contig(start_read, dag, visited, topo_order):
    """overlapGraphs.py:64-103: greedy walk from ``start_read`` to the unvisited successor read that is
    first in topological order, appending each read past the edge's ``end_position``."""
    contig = start_read.split("_")[0]
    visited.add(start_read.split("_")[0])
    neighbors = list(dag.neighbors(start_read))
    while neighbors:
        valid = [nb for nb in neighbors if nb.split("_")[0] not in visited]
        if not valid:
            break
        next_read = min(valid, key=lambda nb: topo_order.get(nb.split("_")[0], float("inf")))
        end = dag.edges[start_read, next_read]["end_position"]
        contig += next_read.split("_")[0][end:]
        start_read = next_read
        neighbors = list(dag.neighbors(start_read))
        visited.add(start_read.split("_")[0])
    return contig


def assemble_contigs_using_overlap_graphs(reads, k=5, params=None, engine: Optional[OverlapEngine] = None,
                                          scorer=None):
    """overlapGraphs.py:151-193: overlap graph (GPU candidates + scoring), cycle removal (native
    replay), topological order, greedy contig walks -- the same contigs in the same order.
    ``params`` (the reference's experiment dict) only feeds the progress lines; ``scorer`` is the
    graph builders' hook for (score, end) from another backend."""
    def say(step):
        if params is not None:
            print(f"{step} for experiment_name={params['experiment_name']} - N={params['N']}, l={params['l']}, "
                  f"p={params['error_prob']}, k={params['k']}, num_iteration={params['num_iteration']}...")
    say("Constructing overlap graph")
    overlap_graph, read_copies = construct_overlap_graph_nx_k(reads, k=k, engine=engine, scorer=scorer)
    say("Removing cycles from graph")
    dag = remove_cycles_from_graph(overlap_graph)
    topo_with_copies = {node: i for i, node in enumerate(nx.topological_sort(dag))}
    topo_order: Dict[str, int] = {}
    for read_with_copy, i in topo_with_copies.items():
        topo_order[read_with_copy.split("_")[0]] = i
    say("Creating contig")
    visited: set = set()
    contigs = []
    for read in topo_order.keys():
        if read not in visited:
            for copy_index in range(read_copies[read]):
                contigs.append(create_contig(f"{read}_{copy_index}", dag, visited, topo_order))
    return contigs


"""Generate tests/golden/*.json from the reference's own Python source.

CONTAINER-ONLY, TEST INFRASTRUCTURE.  Run here (where /root/reference exists):

    python oracle/gen_golden.py

How the reference is executed:
* Numba and Biopython are not installed (ordinary ModuleNotFoundError, not a
  permission denial).  ``numba.njit`` is replaced by the identity decorator and
  ``Bio.Align.PairwiseAligner`` by an unused placeholder (only referenced by
  aligners.py:205-274, off the hot path), so the reference source runs under
  CPython.
* Numba compiles integer arithmetic at int64 (numba/core/typing/builtins.py
  :141-166) and types the omitted ``indel=-2**31`` default as int64.  Under
  CPython + NumPy 2 the same source would do int32 scalar arithmetic and wrap
  (SURVEY.md fact 4), so every call passes the scoring parameters as
  ``np.int64`` to reproduce the Numba typing.  ``construct_overlap_graph_nx_k``
  is run with its module-level ``overlap_alignment`` bound the same way.
* No reference file is copied: only inputs and outputs are written.

Fixtures hold the read strings, so no RNG replay is needed on the GPU box.
"""
from __future__ import annotations

import contextlib
import functools
import io
import json
import os
import random
import sys
import time
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "genome-assembly-using-overlap-graphs_amd"))


def import_reference():
    sys.dont_write_bytecode = True  # never write into /root/reference
    numba = types.ModuleType("numba")

    def njit(*args, **kwargs):
        if len(args) == 1 and callable(args[0]) and not kwargs:
            return args[0]
        return lambda f: f

    numba.njit = njit
    bio = types.ModuleType("Bio")
    align = types.ModuleType("Bio.Align")

    class PairwiseAligner:  # placeholder; the hot path never constructs it
        def __init__(self, *a, **k):
            raise RuntimeError("Biopython is not available")

    align.PairwiseAligner = PairwiseAligner
    bio.Align = align
    sys.modules.setdefault("numba", numba)
    sys.modules.setdefault("Bio", bio)
    sys.modules.setdefault("Bio.Align", align)
    sys.path.insert(0, REF)
    import aligners  # noqa: E402
    import overlapGraphs  # noqa: E402
    import generateErrorFreeReads  # noqa: E402
    return aligners, overlapGraphs, generateErrorFreeReads


def ref_call(aligners, s, t, match=10, mismatch=-1, indel=-(2 ** 31)):
    to_print, a_s, a_t, score, end = aligners.overlap_alignment(
        s, t, match_score=np.int64(match), mismatch=np.int64(mismatch), indel=np.int64(indel))
    return str(to_print), str(a_s), str(a_t), int(score), int(end)


def rand_seq(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def mutate(rng, s, p, alphabet="ACGT"):
    out = []
    for ch in s:
        if rng.random() <= p:
            out.append(rng.choice([c for c in alphabet if c != ch]))
        else:
            out.append(ch)
    return "".join(out)


def default_pairs(rng, genome):
    """Random and realistic pairs under the default scoring (the hot path's regime)."""
    pairs = []
    # edge cases
    edge = [("", ""), ("A", ""), ("", "ACGT"), ("A", "A"), ("A", "C"), ("AC", "CA"), ("ACGT", "ACGT"),
            ("AAAA", "AAAA"), ("ACGTACGT", "GTACGTAA"), ("T" * 40, "T" * 33), ("GATTACA", "TACAGATTACA")]
    pairs += edge
    # word-boundary lengths around multiples of 32 and 64
    for n in (31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 160, 191, 192, 193, 224, 255, 256):
        for m in (n, 1, 32, 64, 100, 129, 256):
            pairs.append((rand_seq(rng, n), rand_seq(rng, m)))
    # random lengths 1..260, unrelated
    for _ in range(300):
        pairs.append((rand_seq(rng, rng.randint(1, 260)), rand_seq(rng, rng.randint(1, 260))))
    # realistic overlaps from the genome (suffix of s == prefix of t, with errors)
    G = len(genome)
    for _ in range(500):
        l = rng.choice([50, 100, 100, 150, 250])
        st = rng.randint(0, G - 1)
        s = genome[st:st + l]
        shift = rng.randint(1, max(1, len(s) - 1))
        t = genome[st + shift: st + shift + l]
        if not t:
            t = rand_seq(rng, l)
        p = rng.choice([0.0, 0.01, 0.02, 0.05])
        pairs.append((mutate(rng, s, p), mutate(rng, t, p)))
    # identical and near-identical
    for _ in range(40):
        s = rand_seq(rng, rng.randint(1, 200))
        pairs.append((s, s))
        pairs.append((s, mutate(rng, s, 0.1)))
    return pairs


def param_pairs(rng, genome):
    """Non-default scoring, including finite gap penalties (gapped DP regime)."""
    params = [(10, -1, -1), (10, -1, -2), (10, -1, -5), (10, -1, -20), (1, -1, -1), (2, -3, -5),
              (5, -4, -8), (1, -2, -2), (3, 1, -1), (10, -1, -100), (10, -1, -(2 ** 31)), (1, 0, 0),
              (-1, 2, -1), (7, -7, -3)]
    out = []
    G = len(genome)
    for (ma, mm, ind) in params:
        for _ in range(36):
            kind = rng.random()
            if kind < 0.5:
                s = rand_seq(rng, rng.randint(0, 60)); t = rand_seq(rng, rng.randint(0, 60))
            else:
                l = rng.randint(8, 60); st = rng.randint(0, G - 1)
                s = genome[st:st + l]
                sh = rng.randint(0, max(0, len(s) - 1))
                t = genome[st + sh: st + sh + l] or rand_seq(rng, l)
                # indels so that gaps can matter
                if rng.random() < 0.5 and len(t) > 3:
                    q = rng.randint(1, len(t) - 2)
                    t = t[:q] + t[q + 1:] if rng.random() < 0.5 else t[:q] + rng.choice("ACGT") + t[q:]
                s = mutate(rng, s, 0.03)
            out.append((s, t, ma, mm, ind))
    return out


def alphabet_pairs(rng):
    out = []
    alphs = ["ACGTN", "acgtACGT", "ACGTRYKMSWBDHVN-", "01", "xyzXYZ#@!", "ACGTé∆"]
    for al in alphs:
        for _ in range(30):
            out.append((rand_seq(rng, rng.randint(0, 120), al), rand_seq(rng, rng.randint(0, 120), al)))
    return out


def graph_record(G, copies, distinct_index):
    """Compact graph encoding: node names -> (distinct-read index, copy)."""
    def enc(name):
        read, _, cp = name.rpartition("_")
        return [distinct_index[read], int(cp)]
    nodes = [enc(n) for n in G.nodes()]
    edges = [enc(u) + enc(v) + [int(d["weight"]), int(d["end_position"])] for u, v, d in G.edges(data=True)]
    # predecessor order per node pins the global edge insertion order (G.edges() only shows successors)
    pred = [[enc(p) for p in G.pred[n]] for n in G.nodes()]
    return {"nodes": nodes, "edges": edges, "pred": pred,
            "read_copies": [[distinct_index[r], int(c)] for r, c in copies.items()]}


def graph_case(overlapGraphs, fn_name, reads, **kw):
    fn = getattr(overlapGraphs, fn_name)
    with contextlib.redirect_stdout(io.StringIO()):
        res = fn(reads, **kw)
    distinct = list(dict.fromkeys(reads))
    idx = {r: i for i, r in enumerate(distinct)}
    if isinstance(res, tuple):
        G, copies = res
    else:  # construct_string_graph returns only the graph; nodes are raw reads
        G, copies = res, None
    if fn_name == "construct_string_graph":
        nodes = [idx[n] for n in G.nodes()]
        edges = [[idx[u], idx[v], int(d["weight"]), int(d["end_position"])] for u, v, d in G.edges(data=True)]
        pred = [[idx[p] for p in G.pred[n]] for n in G.nodes()]
        rec = {"nodes": nodes, "edges": edges, "pred": pred}
    else:
        rec = graph_record(G, copies, idx)
    rec.update({"fn": fn_name, "kwargs": kw, "reads": list(reads), "distinct": distinct})
    return rec


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    aligners, overlapGraphs, gefr = import_reference()
    overlapGraphs.overlap_alignment = functools.partial(
        aligners.overlap_alignment, indel=np.int64(-(2 ** 31)))
    genome = gefr.read_genome_from_fasta(os.path.join(REF, "sequence.fasta"))
    rng = random.Random(20261015)
    meta = {"generator": "oracle/gen_golden.py", "reference": "roiteichman/Genome-Assembly-Using-Overlap-Graphs",
            "numba": "absent: njit replaced by identity; scoring args passed as np.int64 (Numba int64 typing)"}

    t0 = time.time()
    recs = []
    for i, (s, t) in enumerate(default_pairs(rng, genome)):
        tp, a_s, a_t, sc, en = ref_call(aligners, s, t)
        rec = {"s": s, "t": t, "score": sc, "end": en}
        if i % 5 == 0 or len(s) <= 40:
            rec.update({"to_print": tp, "align_s": a_s, "align_t": a_t})
        recs.append(rec)
    with open(os.path.join(GOLDEN, "pairs_default.json"), "w") as fh:
        json.dump({"meta": meta, "params": [10, -1, -(2 ** 31)], "pairs": recs}, fh)
    print(f"pairs_default: {len(recs)} pairs in {time.time() - t0:.1f}s")

    t0 = time.time()
    recs = []
    for (s, t, ma, mm, ind) in param_pairs(rng, genome):
        tp, a_s, a_t, sc, en = ref_call(aligners, s, t, ma, mm, ind)
        recs.append({"s": s, "t": t, "match": ma, "mismatch": mm, "indel": ind, "score": sc, "end": en,
                     "to_print": tp, "align_s": a_s, "align_t": a_t})
    with open(os.path.join(GOLDEN, "pairs_params.json"), "w") as fh:
        json.dump({"meta": meta, "pairs": recs}, fh)
    print(f"pairs_params: {len(recs)} pairs in {time.time() - t0:.1f}s")

    t0 = time.time()
    recs = []
    for (s, t) in alphabet_pairs(rng):
        tp, a_s, a_t, sc, en = ref_call(aligners, s, t)
        recs.append({"s": s, "t": t, "score": sc, "end": en, "to_print": tp, "align_s": a_s, "align_t": a_t})
    with open(os.path.join(GOLDEN, "pairs_alphabet.json"), "w", encoding="utf-8") as fh:
        json.dump({"meta": meta, "pairs": recs}, fh, ensure_ascii=False)
    print(f"pairs_alphabet: {len(recs)} pairs in {time.time() - t0:.1f}s")

    # graphs --------------------------------------------------------------
    t0 = time.time()
    graphs = []
    random.seed(0)
    cfg1 = gefr.generate_error_free_reads(genome, 100, 500)  # BASELINE configs[0]
    graphs.append(dict(graph_case(overlapGraphs, "construct_overlap_graph_nx_k", cfg1, k=5), name="cfg1"))
    grng = random.Random(7)
    region = genome[1000:1400]
    small = [region[st:st + 30] for st in (grng.randint(0, 380) for _ in range(36))]
    small += [small[0], small[0], small[3], "ACG", "ACGTA", region[390:]]  # copies, short reads, tail read
    small_err = [mutate(grng, r, 0.05) for r in small]
    for k in (0, 1, 3, 5, 10):
        graphs.append(dict(graph_case(overlapGraphs, "construct_overlap_graph_nx_k", small, k=k), name=f"small_k{k}"))
    graphs.append(dict(graph_case(overlapGraphs, "construct_overlap_graph_nx_k", small_err, k=4), name="small_err_k4"))
    random.seed(1)
    mid = gefr.generate_error_free_reads(genome, 60, 300)
    mid = [mutate(grng, r, 0.01) for r in mid]
    graphs.append(dict(graph_case(overlapGraphs, "construct_overlap_graph_nx_k", mid, k=5), name="mid_p01_k5"))
    graphs.append(dict(graph_case(overlapGraphs, "construct_overlap_graph_string", small[:20]), name="string_small"))
    graphs.append(dict(graph_case(overlapGraphs, "construct_string_graph", small[:20] + small[:2]), name="stringgraph_small"))
    with open(os.path.join(GOLDEN, "graphs.json"), "w") as fh:
        json.dump({"meta": meta, "graphs": graphs}, fh)
    print(f"graphs: {len(graphs)} graphs in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()

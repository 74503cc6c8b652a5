"""Generate tests/golden/local_alignment.json from the reference's own local_alignment source.

CONTAINER-ONLY, TEST INFRASTRUCTURE.  Run here (where /root/reference exists):

    python oracle/gen_golden_local.py

Executes aligners.local_alignment (aligners.py:85-167) and
aligners.align_read_or_contig_to_reference (aligners.py:170-202) exactly as
oracle/gen_golden.py executes overlap_alignment: numba.njit replaced by the
identity, scoring arguments passed as np.int64 (Numba's int64 typing).  Only
inputs and outputs are written.
"""
from __future__ import annotations

import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import GOLDEN, REF, import_reference, mutate, rand_seq  # noqa: E402


def indel_mutate(rng, s, p_sub, p_indel):
    out = []
    for ch in s:
        u = rng.random()
        if u < p_indel / 2:
            continue
        if u < p_indel:
            out.append(rng.choice("ACGT"))
        out.append(rng.choice([c for c in "ACGT" if c != ch]) if rng.random() < p_sub else ch)
    return "".join(out)


def main():
    aligners, _, gefr = import_reference()
    genome = gefr.read_genome_from_fasta(os.path.join(REF, "sequence.fasta"))
    rng = random.Random(20261016)
    G = len(genome)

    def call(q, r, ma, mm, ind):
        tp, a_r, a_q, sc, st, en = aligners.local_alignment(q, r, np.int64(ma), np.int64(mm), np.int64(ind))
        return {"query": q, "reference": r, "match": ma, "mismatch": mm, "indel": ind, "to_print": str(tp),
                "aligned_reference": str(a_r), "aligned_query": str(a_q), "score": int(sc), "start": int(st),
                "end": int(en)}

    t0 = time.time()
    recs = []
    edge = [("", ""), ("A", ""), ("", "ACGT"), ("A", "A"), ("A", "C"), ("AC", "CA"), ("ACGT", "ACGT"),
            ("AAAA", "AAAAAAAA"), ("GATTACA", "TACAGATTACA"), ("ACGTACGT", "TTTTTTTT"), ("T" * 40, "T" * 33)]
    for q, r in edge:
        recs.append(call(q, r, 10, -1, -1))
    params = [(10, -1, -1), (1, -1, -1), (2, -3, -5), (5, -4, -8), (10, -1, -20), (1, 0, 0), (3, -1, -2),
              (1, -2, -1)]
    for (ma, mm, ind) in params:
        for _ in range(30):
            if rng.random() < 0.4:
                q, r = rand_seq(rng, rng.randint(0, 70)), rand_seq(rng, rng.randint(0, 90))
            else:
                st = rng.randint(0, G - 1)
                r = genome[st:st + rng.randint(10, 90)]
                q = indel_mutate(rng, r[rng.randint(0, max(0, len(r) - 5)):], 0.05, 0.05)
                if rng.random() < 0.5:
                    q = rand_seq(rng, rng.randint(0, 10)) + q + rand_seq(rng, rng.randint(0, 10))
            recs.append(call(q, r, ma, mm, ind))
    # reads against genome windows (the evaluation path's shape, scaled down)
    for _ in range(40):
        st = rng.randint(0, G - 400)
        window = genome[st:st + rng.randint(150, 400)]
        off = rng.randint(0, len(window) - 50)
        q = indel_mutate(rng, window[off:off + rng.randint(30, 120)], 0.02, 0.02)
        recs.append(call(q, window, 10, -1, -1))
    # one larger contig-vs-window case (multiple 64-row strips and 64-column chunks)
    st = rng.randint(0, G - 1600)
    window = genome[st:st + 1500]
    contig = indel_mutate(rng, window[200:700], 0.01, 0.01)
    recs.append(call(contig, window, 10, -1, -1))
    print(f"local_alignment: {len(recs)} pairs in {time.time() - t0:.1f}s")

    t0 = time.time()
    arc = []
    for _ in range(20):
        read_length = rng.choice([50, 100])
        st = rng.randint(0, G - 300)
        ref = genome[st:st + 300]
        if rng.random() < 0.5:
            item = indel_mutate(rng, ref[-rng.randint(10, read_length - 1):], 0.03, 0.02)  # shorter: tail path
        else:
            o = rng.randint(0, 150)
            item = indel_mutate(rng, ref[o:o + rng.randint(read_length, 150)], 0.03, 0.02)
        tp, a_r, a_q, sc, s0, e0 = aligners.align_read_or_contig_to_reference(
            item, ref, read_length, np.int64(10), np.int64(-1), np.int64(-1))
        arc.append({"item": item, "reference": ref, "read_length": read_length, "to_print": str(tp),
                    "aligned_reference": str(a_r), "aligned_query": str(a_q), "score": int(sc), "start": int(s0),
                    "end": int(e0)})
    print(f"align_read_or_contig_to_reference: {len(arc)} cases in {time.time() - t0:.1f}s")
    meta = {"generator": "oracle/gen_golden_local.py", "reference": "roiteichman/Genome-Assembly-Using-Overlap-Graphs",
            "numba": "absent: njit replaced by identity; scoring args passed as np.int64 (Numba int64 typing)"}
    with open(os.path.join(GOLDEN, "local_alignment.json"), "w") as fh:
        json.dump({"meta": meta, "pairs": recs, "align_to_reference": arc}, fh)


if __name__ == "__main__":
    main()

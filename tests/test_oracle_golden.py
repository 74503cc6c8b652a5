"""The oracle (CPU restatement) pinned against the golden vectors from the reference source."""
import numpy as np
import pytest

from conftest import assert_graph_matches_record


def test_c_dp_matches_golden_default(golden_default, oracle_mod):
    pairs = golden_default["pairs"]
    reads = []
    for p in pairs:
        reads += [p["s"], p["t"]]
    a = np.arange(0, len(reads), 2, dtype=np.int32)
    b = a + 1
    sc, en = oracle_mod.batch_dp(reads, a, b)
    assert sc.tolist() == [p["score"] for p in pairs]
    assert en.tolist() == [p["end"] for p in pairs]


def test_closed_form_matches_golden_default(golden_default, oracle_mod):
    pairs = golden_default["pairs"]
    reads = []
    for p in pairs:
        reads += [p["s"], p["t"]]
    a = np.arange(0, len(reads), 2, dtype=np.int32)
    sc, en = oracle_mod.batch_ungapped(reads, a, a + 1)
    assert sc.tolist() == [p["score"] for p in pairs]
    assert en.tolist() == [p["end"] for p in pairs]
    # and the pure-Python closed form on a slice
    for p in pairs[:60]:
        assert oracle_mod.ungapped(p["s"], p["t"]) == (p["score"], p["end"])


def test_python_restatement_full_tuple(golden_default, golden_params, golden_alphabet, oracle_mod):
    n = 0
    for p in golden_default["pairs"]:
        if "to_print" in p and len(p["s"]) * len(p["t"]) <= 20000:
            got = oracle_mod.overlap_alignment(p["s"], p["t"])
            assert list(got) == [p["to_print"], p["align_s"], p["align_t"], p["score"], p["end"]]
            n += 1
    for p in golden_params["pairs"]:
        got = oracle_mod.overlap_alignment(p["s"], p["t"], p["match"], p["mismatch"], p["indel"])
        assert list(got) == [p["to_print"], p["align_s"], p["align_t"], p["score"], p["end"]]
        n += 1
    for p in golden_alphabet["pairs"]:
        got = oracle_mod.overlap_alignment(p["s"], p["t"])
        assert list(got) == [p["to_print"], p["align_s"], p["align_t"], p["score"], p["end"]]
        n += 1
    assert n > 700


def test_c_dp_matches_golden_params(golden_params, oracle_mod):
    for p in golden_params["pairs"]:
        assert oracle_mod.dp_one(p["s"], p["t"], p["match"], p["mismatch"], p["indel"]) == (p["score"], p["end"])


def test_gapped_cases_really_use_gaps(golden_params):
    # the params fixture must exercise the gapped regime, not only diagonals
    gapped = [p for p in golden_params["pairs"] if "-" in p["align_s"] or "-" in p["align_t"]]
    assert len(gapped) > 30


def test_c_dp_matches_golden_alphabet(golden_alphabet, oracle_mod):
    for p in golden_alphabet["pairs"]:
        assert oracle_mod.dp_one(p["s"], p["t"]) == (p["score"], p["end"])


def test_gaps_cannot_win_condition(golden_params, oracle_mod):
    # whenever the condition holds, the closed form equals the reference DP
    for p in golden_params["pairs"]:
        lmax = max(len(p["s"]), len(p["t"]), 1)
        if oracle_mod.gaps_cannot_win(p["match"], p["mismatch"], p["indel"], lmax):
            sc, en = oracle_mod.ungapped(p["s"], p["t"], p["match"], p["mismatch"])
            assert (sc, en) == (p["score"], p["end"])


def test_graph_restatement_matches_golden(golden_graphs, oracle_mod):
    for rec in golden_graphs["graphs"]:
        if rec["fn"] != "construct_overlap_graph_nx_k":
            continue
        G, copies = oracle_mod.graph_nx_k(rec["reads"], **rec["kwargs"])
        assert_graph_matches_record(G, rec, copies)


def test_int32_wrap_semantics(oracle_mod):
    # stores wrap to int32 like Numba's int32 table (aligners.py:28 + int64 arithmetic)
    big = 2 ** 30
    s, t = "AAAA", "AAAA"
    py = oracle_mod.overlap_alignment(s, t, big, -1, -(2 ** 40))
    c = oracle_mod.dp_one(s, t, big, -1, -(2 ** 40))
    assert (py[3], py[4]) == c


def test_local_alignment_oracle_matches_golden(oracle_mod):
    """oracle_local_align (C) + string rebuild == the reference's local_alignment and
    align_read_or_contig_to_reference outputs (tests/golden/local_alignment.json)."""
    from conftest import load_golden
    d = load_golden("local_alignment.json")
    for rec in d["pairs"]:
        got = oracle_mod.local_alignment(rec["query"], rec["reference"], rec["match"], rec["mismatch"], rec["indel"])
        assert got == (rec["to_print"], rec["aligned_reference"], rec["aligned_query"], rec["score"], rec["start"],
                       rec["end"])
    for rec in d["align_to_reference"]:
        got = oracle_mod.align_read_or_contig_to_reference(rec["item"], rec["reference"], rec["read_length"])
        assert got == (rec["to_print"], rec["aligned_reference"], rec["aligned_query"], rec["score"], rec["start"],
                       rec["end"])

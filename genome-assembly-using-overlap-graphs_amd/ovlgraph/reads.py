"""Genome loading and deterministic read simulation for the benchmark configs.

This is host-side workload generation, not the hot path. It reproduces the
*distribution* of the reference simulator so that candidate-pair counts and
read-length mixes match BASELINE.json's configs:

* ``read_genome_from_fasta`` follows ``generateErrorFreeReads.py:4-19``:
  header lines (``>``) are skipped and the remaining lines are stripped and
  concatenated.
* ``simulate_reads`` follows ``generateErrorFreeReads.py:22-52`` (start uniform
  in ``[0, G-1]``, read truncated at the genome end, never cyclic) and
  ``generateErrorProneReads.py:4-28`` (each base substituted when
  ``U <= p``; the substitute is uniform over the other three bases, using the
  alphabet table of ``generateErrorProneReads.py:43``).

The reference draws from Python ``random`` and Numba's ``np.random`` stream,
which cannot be replayed here, so the stream is numpy PCG64 seeded per config.
Parity never depends on the RNG: golden fixtures embed the read strings.
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

_DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
PHIX_FASTA = os.path.join(_DATA_DIR, "phix174_NC_001422.fasta")

_BASES = np.frombuffer(b"ACGT", dtype=np.uint8)
# generateErrorProneReads.py:43 -> {"A": "CGT", "C": "AGT", "G": "ACT", "T": "ACG"}
_SUBST = {ord("A"): b"CGT", ord("C"): b"AGT", ord("G"): b"ACT", ord("T"): b"ACG"}


def read_genome_from_fasta(path: str = PHIX_FASTA) -> str:
    """Concatenate the sequence lines of a FASTA file (generateErrorFreeReads.py:4-19)."""
    parts = []
    with open(path, "r") as fh:
        for line in fh:
            if not line.startswith(">"):
                parts.append(line.strip())
    return "".join(parts)


def random_genome(length: int, seed: int = 0) -> str:
    """A uniform iid-ACGT genome (cfg4's synthetic 1 Mbp genome)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    return _BASES[rng.integers(0, 4, size=length)].tobytes().decode("ascii")


def simulate_reads(genome: str, read_length: int, num_reads: int, error_prob: float = 0.0,
                   seed: int = 0) -> List[str]:
    """Sample ``num_reads`` reads of length ``read_length`` and add substitution errors.

    Start positions are uniform on ``[0, G-1]``; a read starting within
    ``read_length`` of the end is truncated there (generateErrorFreeReads.py:44-48).
    Each base is substituted with probability ``error_prob`` (``U <= p``,
    generateErrorProneReads.py:16) by a uniformly chosen different base.
    """
    if read_length <= 0 or num_reads < 0:
        raise ValueError("read_length must be > 0 and num_reads >= 0")
    g = np.frombuffer(genome.encode("ascii"), dtype=np.uint8)
    G = g.shape[0]
    rng = np.random.Generator(np.random.PCG64(seed))
    starts = rng.integers(0, G, size=num_reads)
    out: List[str] = []
    # substitution lookup: (base, choice 0..2) -> new base
    sub = np.zeros((256, 3), dtype=np.uint8)
    for b, alts in _SUBST.items():
        sub[b] = np.frombuffer(alts, dtype=np.uint8)
    for st in starts.tolist():
        end = min(st + read_length, G)
        r = g[st:end].copy()
        if error_prob > 0.0:
            u = rng.random(r.shape[0])
            pos = np.nonzero(u <= error_prob)[0]
            if pos.size:
                choice = rng.integers(0, 3, size=pos.size)
                r[pos] = sub[r[pos], choice]
        out.append(r.tobytes().decode("ascii"))
    return out


# Named workloads from BASELINE.json "configs" (SURVEY.md §8d).
CONFIGS = {
    "cfg1": dict(genome="phix", N=500, l=100, p=0.0, k=5),
    "cfg2": dict(genome="phix", N=10_000, l=100, p=0.01, k=5),
    "cfg3": dict(genome="phix", N=50_000, l=150, p=0.02, k=5),
    "cfg4": dict(genome="random1M", N=200_000, l=100, p=0.01, k=5),
    "cfg5": dict(genome="phix", N=50_000, l=250, p=0.05, k=5),
    "target": dict(genome="phix", N=50_000, l=100, p=0.01, k=5),
}


def config_reads(name: str, seed: int = 0, genome: Optional[str] = None) -> List[str]:
    """Reads for a named config (seeded)."""
    c = CONFIGS[name]
    if genome is None:
        genome = read_genome_from_fasta() if c["genome"] == "phix" else random_genome(1_000_000, seed=1234)
    return simulate_reads(genome, c["l"], c["N"], c["p"], seed=seed)

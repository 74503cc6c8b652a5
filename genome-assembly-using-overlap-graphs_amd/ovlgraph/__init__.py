"""ovlgraph — MI355X-native drop-in for the overlap-scoring path of
roiteichman/Genome-Assembly-Using-Overlap-Graphs (aligners.py / overlapGraphs.py).

    from ovlgraph.overlapGraphs import construct_overlap_graph_nx_k
    from ovlgraph.aligners import overlap_alignment

Candidate pairs are enumerated on the host (Python), every pair is scored by
hand-written gfx950 HIP kernels behind the C ABI of include/ovl.h.
"""
from ._lib import OvlError  # noqa: F401
from .engine import INDEL_DEFAULT, OverlapEngine, default_engine, encode_reads, score_reads  # noqa: F401

__all__ = ["OvlError", "OverlapEngine", "default_engine", "encode_reads", "score_reads", "INDEL_DEFAULT"]

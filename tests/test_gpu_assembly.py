"""The assembly pipeline drop-in on the GPU path: assemble_contigs_using_overlap_graphs
(overlapGraphs.py:151-193) with device candidates and GPU scoring gives the reference's contigs
(tests/golden/assembly.json, from the reference function)."""
import contextlib
import io

import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_assembly_pipeline_gpu_matches_reference_contigs():
    from ovlgraph import overlapGraphs as og
    for case in load_golden("assembly.json")["cases"]:
        with contextlib.redirect_stdout(io.StringIO()):
            contigs = og.assemble_contigs_using_overlap_graphs(case["reads"], k=case["k"], params=case["params"])
        assert contigs == case["contigs"]

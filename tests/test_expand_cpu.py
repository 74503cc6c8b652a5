"""CPU: the host expansion of packed results (csrc/ovl_expand.h: the scalar form and its SSE2 / AVX2 /
AVX-512 variants) on random packed entries -- normal, escaped (score stored separately) and bad pairs --
at every destination alignment and range; tests/c/expand_test.cpp compares each variant this CPU runs with
the scalar form."""
import os
import subprocess

from conftest import PKG, ROOT


def test_expand_variants_match_scalar(tmp_path):
    exe = tmp_path / "expand_test"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(PKG, "csrc"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "c", "expand_test.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "ok"
    assert "checked sse2" in lines


def test_tile_records_decode(tmp_path):
    """The tile records of the resident grid's ring (ovl_kernels.hip put_ring_rec: 15-bit codes j(j + 1)/2 + X and
    a phase bit per dword, special words apart; the decoders' side-array form): tests/c/rec_test.cpp checks every code, random tiles in both phases
    through the scalar and (where this CPU runs it) AVX-512 decoders, the readiness test on incomplete records,
    the special words each decode reports for zeroing, and a special word that has not landed."""
    exe = tmp_path / "rec_test"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(PKG, "csrc"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "c", "rec_test.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "ok" and lines[0] == "checked codes", lines

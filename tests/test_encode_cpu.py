"""CPU: the host encoding of compact pair lists (csrc/ovl_encode.h: b narrowed to uint16, the runs of an
a-major list) -- tests/c/encode_test.cpp compares each vector variant this CPU runs (AVX2, AVX-512) with the
scalar form over a-major and unsorted lists, out-of-range indices, run caps and unaligned outputs."""
import os
import subprocess

from conftest import PKG, ROOT


def test_encode_variants_match_scalar(tmp_path):
    exe = tmp_path / "encode_test"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(PKG, "csrc"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "c", "encode_test.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "ok"
    assert any(x.startswith("checked") for x in lines) or all(x.startswith("skip") for x in lines[:-1])


def test_read_scan_pack_matches_scalar(tmp_path):
    """csrc/ovl_scan.h: the read-set scan with 2-bit packing (ovl_set_reads' upload of ACGT-only bytes), the
    AVX-512 form against the scalar one and a direct restatement (tests/c/scan_test.cpp)."""
    exe = tmp_path / "scan_test"
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(PKG, "csrc"),
                        "-o", str(exe), os.path.join(ROOT, "tests", "c", "scan_test.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.splitlines()
    assert lines[-1] == "ok" and "checked scalar" in lines

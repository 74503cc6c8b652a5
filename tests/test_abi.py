"""The C-ABI library loads and exports exactly what include/ovl.h declares (no GPU compute)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from ovlgraph import _lib

HEADER = os.path.join(ROOT, "include", "ovl.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ovl_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_surface():
    names = declared_functions()
    assert names == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (ovl_[a-z_]+)", out)))
    assert exported == declared_functions()  # nothing else leaks (launchers are hidden)


def test_version():
    assert _lib.load().ovl_version() == _lib.ABI_VERSION


def test_null_args_are_errors_not_crashes():
    L = _lib.load()
    assert L.ovl_device_count(None) == -1
    assert L.ovl_create(0, None) == -1
    assert L.ovl_set_reads(None, None, None, 0) == -1
    assert L.ovl_score_host(None, None, None, 0, 10, -1, -(2 ** 31), -1, None, None) == -1
    assert L.ovl_quiesce(None) == -1
    assert L.ovl_resident_stats(None, None, None, None, None) == -1
    assert L.ovl_devices_for(None, 10, None) == -1
    assert L.ovl_destroy(None) == 0
    assert isinstance(_lib.last_error(None), str)


def test_built_for_gfx950_only():
    blob = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ovlgraph import OverlapEngine, OvlError
    with pytest.raises(OvlError):
        OverlapEngine(-1)

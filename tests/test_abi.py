"""C-ABI boundary checks that need no GPU: the shared library loads and
exports exactly what include/rifraf_hip.h declares; without a device the
engine refuses loudly instead of falling back to the CPU."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rifraf_hip.h")
LIB = os.path.join(REPO, "rifraf.jl_amd", "librifraf_hip.so")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rf_\w+)\s*\(", text, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ["rf_create", "rf_destroy", "rf_last_error", "rf_set_sequences", "rf_set_templates",
              "rf_realign", "rf_backtrace", "rf_score", "rf_download_band", "rf_slot_geometry"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.fail("librifraf_hip.so not built: run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB)
    for s in declared_symbols():
        assert hasattr(lib, s), f"missing export {s}"


def test_binding_signatures_cover_header():
    from rifraf_amd import _lib
    assert set(_lib._SIGNATURES) == set(declared_symbols())
    lib = _lib.load()
    assert lib.rf_abi_version() == _lib.RF_ABI_VERSION


def test_no_device_is_loud():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from rifraf_amd._lib import EngineUnavailable
    from rifraf_amd.engine import Engine
    with pytest.raises(EngineUnavailable):
        Engine(0)


def test_missing_library_is_loud(tmp_path):
    from rifraf_amd import _lib
    with pytest.raises(_lib.EngineUnavailable):
        _lib.load(str(tmp_path / "nope.so"))

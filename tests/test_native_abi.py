"""The C ABI boundary without a GPU: libncgpu.so loads, exports every symbol
include/ncgpu.h declares, and the ctypes binding agrees with each prototype's
arity (a mismatch silently truncates pointers — caught here, not on the GPU)."""
import re
from pathlib import Path

import pytest

from nightcore_analyzer import _native

HEADER = Path(__file__).resolve().parents[1] / "include" / "ncgpu.h"


def _prototypes():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(?:int|size_t|const char\s*\*)\s+(nc_\w+)\s*\(([^;]*?)\)\s*;", text, flags=re.S):
        args = m.group(2).strip()
        protos[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return protos


def test_header_parses():
    p = _prototypes()
    assert len(p) >= 25 and "nc_window_stage" in p and "nc_bootstrap_ratio" in p


def test_library_exports_every_declared_symbol():
    if not _native.lib_path().exists():
        pytest.skip("libncgpu.so not built (run __graft_entry__.build())")
    lib = _native.load()
    missing = [n for n in _prototypes() if getattr(lib, n, None) is None]
    assert not missing, missing


def test_ctypes_signatures_match_prototypes():
    protos = _prototypes()
    assert set(protos) == set(_native.SIGNATURES), set(protos) ^ set(_native.SIGNATURES)
    for name, n in protos.items():
        assert len(_native.SIGNATURES[name][1]) == n, (name, n, len(_native.SIGNATURES[name][1]))


def test_abi_version_and_loud_failure_without_device():
    if not _native.lib_path().exists():
        pytest.skip("libncgpu.so not built")
    import torch
    lib = _native.load()
    assert lib.nc_abi_version() == 5
    if torch.cuda.is_available():
        pytest.skip("a device is visible; the no-device path is exercised on CPU hosts")
    with pytest.raises(_native.NativeUnavailable):
        _native.Context(0)

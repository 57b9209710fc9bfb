"""C ABI checks that need no GPU: every symbol include/clay.h declares is exported
by libclay_amd.so and bound in clay_amd._lib; struct layouts agree; the product
refuses to compute without a device (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

from clay_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "clay.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(clay_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_api():
    names = declared_functions()
    for n in ("clay_new", "clay_new_default", "clay_encode", "clay_decode", "clay_minimum_to_repair",
              "clay_repair", "clay_normalized_repair_bandwidth", "clay_encode_device",
              "clay_decode_device", "clay_repair_device"):
        assert n in names


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), f"{name} declared in clay.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} not bound in clay_amd._lib"
    assert set(_lib.SIGNATURES) == set(declared_functions())


def test_library_is_gfx950_hip_binary():
    path = _lib.LIB_PATH
    blob = open(path, "rb").read()
    assert b"gfx950" in blob, "no gfx950 code object in libclay_amd.so"
    assert b"k_fused_encode" in blob and b"k_exec" in blob
    assert _lib.lib().clay_abi_version() == 1


def test_error_struct_layout_matches_oracle(oracle_mod):
    assert C.sizeof(_lib.ClayErrorStruct) == C.sizeof(oracle_mod.OcError)
    assert C.sizeof(_lib.ClayCodeStruct) == C.sizeof(oracle_mod.OcCode) == 11 * 8


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible here")
    from clay_amd import ClayCode, DeviceError
    c = ClayCode(4, 2, 5)
    with pytest.raises(DeviceError):
        c.encode(b"needs a GPU")
    with pytest.raises(DeviceError):
        c.encode_device([1] * 4, [2] * 2, 16)

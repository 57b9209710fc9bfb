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


SHIPPING_KERNELS = {"k_stream_encode", "k_stream_local", "k_stream_local256", "k_stream_fused2", "k_stream_encode3", "k_bs_repair",
                    "k_bs_repair_stream", "k_bs_encode", "k_bs_encode1", "k_bs_decode1", "k_fused_encode", "k_gexec", "k_texec",
                    "k_ygroup"}


def kernel_names(blob: bytes):
    """Kernel names in the embedded gfx950 code object (Itanium-mangled `<len><name>`)."""
    names = set()
    for m in re.finditer(rb"(\d+)(k_[a-z0-9_]+)", blob):
        n = int(m.group(1)[-2:]) if len(m.group(1)) > 1 and int(m.group(1)[-2:]) <= len(m.group(2)) else int(m.group(1)[-1:])
        if n == len(m.group(2)):
            names.add(m.group(2).decode())
    return names


def test_library_is_gfx950_hip_binary():
    path = _lib.LIB_PATH
    blob = open(path, "rb").read()
    assert b"gfx950" in blob, "no gfx950 code object in libclay_amd.so"
    assert _lib.lib().clay_abi_version() == 4


def test_library_ships_only_parity_producing_kernels():
    """Measurement probes and superseded encode variants live in bench_tools/ (their own
    binaries), never in the product library: every kernel in libclay_amd.so is one that
    produces the reference's bytes (tests/test_gpu_parity.py checks each against the oracle)."""
    names = kernel_names(open(_lib.LIB_PATH, "rb").read())
    assert SHIPPING_KERNELS <= names, SHIPPING_KERNELS - names
    assert names <= SHIPPING_KERNELS, names - SHIPPING_KERNELS


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


def test_exec_modes_only_choose_kernels():
    """Retired modes are rejected: 4 (the round-3 single-launch decode) and 7 (the process-wide
    "codeword" mode, which changed the bytes concurrent decodes returned; now the per-call
    clay_decode_device_codeword).  No GPU needed: the setter is host state."""
    import clay_amd
    L = _lib.lib()
    assert L.clay_set_exec_mode(4) == -1 and L.clay_set_exec_mode(7) == -1
    for name in ("codeword", "stream-fused"):
        with pytest.raises(ValueError):
            clay_amd.set_exec_mode(name)
    prev = clay_amd.set_exec_mode("stream")
    assert clay_amd.set_exec_mode(prev) == "stream"
    assert L.clay_set_encode_path(4) == -1  # the retired v6 encode
    with pytest.raises(ValueError):
        clay_amd.set_encode_path("bitsliced6")

"""ctypes binding of include/clay.h (libclay_amd.so, built in-tree).

There is no CPU fallback: if the shared library is missing this module raises
ImportError, and compute calls without a GPU return CLAY_ERR_DEVICE.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CLAY_AMD_LIB selects another build of the same library (the sanitizer build of
# scripts/asan_check.sh); it is never a fallback: a missing library still raises.
LIB_PATH = os.environ.get("CLAY_AMD_LIB") or os.path.join(_HERE, "libclay_amd.so")

CLAY_ERR_DEVICE = 100


class ClayCodeStruct(C.Structure):
    _fields_ = [(n, C.c_size_t) for n in
                ("k", "m", "n", "d", "q", "t", "nu", "sub_chunk_no", "beta",
                 "original_count", "recovery_count")]


class ClayErrorStruct(C.Structure):
    _fields_ = [("kind", C.c_int), ("a", C.c_size_t), ("b", C.c_size_t),
                ("c", C.c_size_t), ("msg", C.c_char * 256)]


# every symbol include/clay.h declares, with (restype, argtypes)
_sz, _P, _u8p, _vp = C.c_size_t, C.POINTER, C.POINTER(C.c_uint8), C.c_void_p
_code_p, _err_p = _P(ClayCodeStruct), _P(ClayErrorStruct)
SIGNATURES = {
    "clay_new": (C.c_int, [_sz, _sz, _sz, _code_p, _err_p]),
    "clay_new_default": (C.c_int, [_sz, _sz, _code_p, _err_p]),
    "clay_normalized_repair_bandwidth": (C.c_double, [_code_p]),
    "clay_encoded_chunk_size": (_sz, [_code_p, _sz]),
    "clay_encode": (C.c_int, [_code_p, _u8p, _sz, _P(_u8p), _sz, _err_p]),
    "clay_decode": (C.c_int, [_code_p, _P(_sz), _P(_u8p), _P(_sz), _sz, _P(_sz), _sz, _u8p, _sz,
                              _P(_sz), _err_p]),
    "clay_minimum_to_repair": (C.c_int, [_code_p, _sz, _P(_sz), _sz, _P(_sz), _P(_sz), _P(_sz),
                                         _P(_sz), _err_p]),
    "clay_repair": (C.c_int, [_code_p, _sz, _P(_sz), _P(_u8p), _P(_sz), _sz, _sz, _u8p, _err_p]),
    "clay_encode_device": (C.c_int, [_code_p, _P(_vp), _P(_vp), _sz, C.c_int, _vp, _err_p]),
    "clay_encode_device_batch": (C.c_int, [_code_p, _P(_vp), _P(_vp), _sz, _sz, C.c_int, _vp,
                                           _err_p]),
    "clay_encode_host_pipelined": (C.c_int, [_code_p, _P(_vp), _P(_vp), _sz, C.c_int, _sz, C.c_int,
                                             _err_p]),
    "clay_decode_device": (C.c_int, [_code_p, _P(_vp), _P(_sz), _sz, _P(_vp), _sz, C.c_int, _vp,
                                     _err_p]),
    "clay_decode_device_codeword": (C.c_int, [_code_p, _P(_vp), _P(_sz), _sz, _P(_vp), _sz, C.c_int, _vp,
                                              _err_p]),
    "clay_repair_device": (C.c_int, [_code_p, _sz, _P(_sz), _P(_vp), _sz, _sz, _vp, C.c_int, _vp,
                                     _err_p]),
    "clay_repair_device_full_chunks": (C.c_int, [_code_p, _sz, _P(_sz), _P(_vp), _sz, _sz, _vp,
                                                 C.c_int, _vp, _err_p]),
    "clay_reserve_workspace": (C.c_int, [_code_p, _sz, C.c_int, _err_p]),
    "clay_release_workspace": (C.c_int, [C.c_int, _err_p]),
    "clay_release_captured": (C.c_int, [C.c_int, _err_p]),
    "clay_chunk_to_ygroup": (C.c_int, [_code_p, _sz, C.c_void_p, C.c_void_p, _sz, C.c_int, C.c_void_p, _err_p]),
    "clay_ygroup_to_chunk": (C.c_int, [_code_p, _sz, C.c_void_p, C.c_void_p, _sz, C.c_int, C.c_void_p, _err_p]),
    "clay_encode_device_strided": (C.c_int, [_code_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                             C.c_int64, _sz, _sz, C.c_int, C.c_void_p, _err_p]),
    "clay_workspace_bytes": (_sz, [C.c_int]),
    "clay_plan_export": (C.c_int, [_code_p, C.c_int, _u8p, _u8p, _sz, _P(C.c_uint32), _sz,
                                   _P(C.c_uint32), _sz, _P(C.c_uint32), _sz, _P(_sz), _err_p]),
    "clay_set_encode_path": (C.c_int, [C.c_int]),
    "clay_set_exec_mode": (C.c_int, [C.c_int]),
    "clay_last_exec_path": (C.c_char_p, []),
    "clay_last_encode_path": (C.c_char_p, []),
    "clay_last_launch_count": (_sz, []),
    "clay_abi_version": (C.c_int, []),
    "clay_build_info": (C.c_char_p, []),
}

_lib = None


def _share_torch_hip_runtime():
    """PyTorch-ROCm ships its own libamdhip64 (same SONAME as /opt/rocm's).  If this
    library loaded first, a later `import torch` would bring up a second HIP runtime
    and torch.cuda would report no device.  Loading torch first makes both bind to one
    runtime, so device pointers and streams from torch are valid here."""
    import importlib.util
    if "torch" not in __import__("sys").modules and importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def lib():
    global _lib
    if _lib is None:
        _share_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"clay_amd: HIP extension {LIB_PATH} is missing -- build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib

"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU restatement (liboracle.so).

The oracle restates the reference path of spool-labs/clay (clay-codes 0.1.2):
encode.rs:30-80, decode.rs:31-576, repair.rs:22-421, transforms.rs:20-161,
coords.rs:30-40, lib.rs:94-259, plus the published algorithm of the
un-vendored dependency reed-solomon-erasure 6.0.0 (see clay_oracle.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
(clay_amd, libclay_amd.so) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CLAY_ORACLE_LIB: the sanitizer build (scripts/asan_check.sh), built by its own make target
_LIB_PATH = os.environ.get("CLAY_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")

ERROR_NAMES = {
    1: "InvalidParameters",
    2: "InsufficientHelpers",
    3: "InvalidChunkSize",
    4: "InsufficientHelperData",
    5: "InconsistentChunkSizes",
    6: "TooManyErasures",
    7: "ReconstructionFailed",
    8: "MissingYSectionHelper",
    9: "Overflow",
}


class OcCode(C.Structure):
    _fields_ = [(n, C.c_size_t) for n in
                ("k", "m", "n", "d", "q", "t", "nu", "sub_chunk_no", "beta",
                 "original_count", "recovery_count")]


class OcError(C.Structure):
    _fields_ = [("kind", C.c_int), ("a", C.c_size_t), ("b", C.c_size_t),
                ("c", C.c_size_t), ("msg", C.c_char * 256)]


class OracleError(Exception):
    def __init__(self, err: OcError):
        self.kind = int(err.kind)
        self.name = ERROR_NAMES.get(self.kind, str(self.kind))
        self.fields = (int(err.a), int(err.b), int(err.c))
        self.msg = err.msg.decode()
        super().__init__(f"{self.name}: {self.msg}")


def _stale(src: str) -> bool:
    return not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)


def build() -> str:
    """Compile liboracle.so (gcc) if missing or stale.  Safe from several processes at once
    (bench ranks, pytest-xdist workers): the check and the make run under an exclusive lock
    on oracle/.build.lock, so one process builds and the others find a fresh library; the
    Makefile also writes the library under a temporary name and renames it into place, so a
    process that loads it never sees a half-written file."""
    src = os.path.join(_HERE, "clay_oracle.c")
    if os.environ.get("CLAY_ORACLE_LIB"):
        return _LIB_PATH
    if not _stale(src):
        return _LIB_PATH
    import fcntl
    with open(os.path.join(_HERE, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if _stale(src):
                subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        sz, P = C.c_size_t, C.POINTER
        u8p = P(C.c_uint8)
        L.oc_gf_mul.restype = C.c_uint8
        L.oc_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.oc_gf_div.restype = C.c_uint8
        L.oc_gf_div.argtypes = [C.c_uint8, C.c_uint8]
        L.oc_gf_add.restype = C.c_uint8
        L.oc_gf_add.argtypes = [C.c_uint8, C.c_uint8]
        L.oc_gf_exp.restype = C.c_uint8
        L.oc_gf_exp.argtypes = [C.c_uint8, sz]
        L.oc_rs_matrix.argtypes = [sz, sz, u8p]
        L.oc_rs_encode.argtypes = [sz, sz, P(u8p), sz]
        L.oc_rs_reconstruct.argtypes = [sz, sz, P(u8p), u8p, sz]
        L.oc_get_plane_vector.argtypes = [sz, sz, sz, P(sz)]
        L.oc_get_companion_layer.restype = sz
        L.oc_get_companion_layer.argtypes = [P(OcCode), sz, sz, sz, sz]
        L.oc_get_max_iscore.restype = sz
        L.oc_get_max_iscore.argtypes = [P(OcCode), P(sz), sz]
        L.oc_checked_pow.argtypes = [sz, sz, P(sz)]
        L.oc_repair_subchunk_indices.argtypes = [P(OcCode), sz, P(sz), P(sz), P(OcError)]
        L.oc_prt.argtypes = [u8p, u8p, u8p, u8p, sz]
        L.oc_pft.argtypes = [u8p, u8p, u8p, u8p, sz]
        L.oc_c_from_u_and_cstar.argtypes = [u8p, u8p, u8p, sz]
        L.oc_u_from_c_and_ustar.argtypes = [u8p, u8p, u8p, sz]
        L.oc_new.argtypes = [sz, sz, sz, P(OcCode), P(OcError)]
        L.oc_new_default.argtypes = [sz, sz, P(OcCode), P(OcError)]
        L.oc_normalized_repair_bandwidth.restype = C.c_double
        L.oc_normalized_repair_bandwidth.argtypes = [P(OcCode)]
        L.oc_encoded_chunk_size.restype = sz
        L.oc_encoded_chunk_size.argtypes = [P(OcCode), sz]
        L.oc_encode.argtypes = [P(OcCode), u8p, sz, u8p, P(OcError)]
        L.oc_decode.argtypes = [P(OcCode), P(sz), P(u8p), P(sz), sz, P(sz), sz, u8p, sz,
                                P(sz), P(OcError)]
        L.oc_minimum_to_repair.argtypes = [P(OcCode), sz, P(sz), sz, P(sz), P(sz), P(sz),
                                           P(sz), P(OcError)]
        L.oc_repair.argtypes = [P(OcCode), sz, P(sz), P(u8p), P(sz), sz, sz, u8p, P(OcError)]
        L.oc_set_simd.argtypes = [C.c_int]
        L.oc_simd_available.restype = C.c_int
        _lib = L
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _sizes(vals):
    arr = (C.c_size_t * max(1, len(vals)))(*[int(v) for v in vals])
    return arr


def _as_np(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8)
    return np.frombuffer(bytes(b), dtype=np.uint8)


# ---- small helpers with reference KATs -------------------------------------
def gf_mul(a, b): return int(lib().oc_gf_mul(a, b))
def gf_div(a, b): return int(lib().oc_gf_div(a, b))
def gf_add(a, b): return int(lib().oc_gf_add(a, b))
def gf_exp(a, n): return int(lib().oc_gf_exp(a, n))
def gf_inv(a): return gf_div(1, a)


def rs_matrix(data: int, parity: int) -> np.ndarray:
    out = np.zeros((data + parity) * data, dtype=np.uint8)
    rc = lib().oc_rs_matrix(data, parity, _u8(out))
    if rc:
        raise ValueError(f"RS init failed ({rc})")
    return out.reshape(data + parity, data)


def rs_encode(data: int, parity: int, shards: list) -> list:
    arrs = [np.array(_as_np(s), copy=True) for s in shards]
    ptrs = (C.POINTER(C.c_uint8) * len(arrs))(*[_u8(a) for a in arrs])
    rc = lib().oc_rs_encode(data, parity, ptrs, arrs[0].size)
    if rc:
        raise ValueError(f"RS encode failed ({rc})")
    return [a.tolist() for a in arrs]


def checked_pow(base: int, exp: int):
    out = C.c_size_t()
    return int(out.value) if lib().oc_checked_pow(base, exp, C.byref(out)) else None


def plane_vector(z: int, t: int, q: int) -> list:
    out = (C.c_size_t * t)()
    lib().oc_get_plane_vector(z, t, q, out)
    return [int(v) for v in out]


def prt(c, cs):
    c, cs = _as_np(c), _as_np(cs)
    u, us = np.zeros_like(c), np.zeros_like(c)
    lib().oc_prt(_u8(c), _u8(cs), _u8(u), _u8(us), c.size)
    return u.tolist(), us.tolist()


def pft(u, us):
    u, us = _as_np(u), _as_np(us)
    c, cs = np.zeros_like(u), np.zeros_like(u)
    lib().oc_pft(_u8(u), _u8(us), _u8(c), _u8(cs), u.size)
    return c.tolist(), cs.tolist()


def c_from_u_and_cstar(u, cs):
    """transforms.rs:132-142: C = U + gamma * C*."""
    u, cs = _as_np(u), _as_np(cs)
    c = np.zeros_like(u)
    lib().oc_c_from_u_and_cstar(_u8(u), _u8(cs), _u8(c), u.size)
    return c.tolist()


def u_from_c_and_ustar(c, us):
    """transforms.rs:149-161: U = det * C + gamma * U*."""
    c, us = _as_np(c), _as_np(us)
    u = np.zeros_like(c)
    lib().oc_u_from_c_and_ustar(_u8(c), _u8(us), _u8(u), c.size)
    return u.tolist()


def set_simd(enable: bool):
    lib().oc_set_simd(1 if enable else 0)


def simd_available() -> bool:
    return bool(lib().oc_simd_available())


class OracleClay:
    """ClayCode (lib.rs:57-242) restated on the CPU -- the checker."""

    def __init__(self, k: int, m: int, d: int):
        self._c = OcCode()
        err = OcError()
        if lib().oc_new(k, m, d, C.byref(self._c), C.byref(err)):
            raise OracleError(err)
        for name, _ in OcCode._fields_:
            setattr(self, name, int(getattr(self._c, name)))

    @classmethod
    def new_default(cls, k: int, m: int) -> "OracleClay":
        return cls(k, m, k + m - 1)

    def max_iscore(self, erased_internal) -> int:
        arr = _sizes(erased_internal)
        return int(lib().oc_get_max_iscore(C.byref(self._c), arr, len(erased_internal)))

    def companion_layer(self, z, x, y, z_y) -> int:
        return int(lib().oc_get_companion_layer(C.byref(self._c), z, x, y, z_y))

    def repair_subchunk_indices(self, lost_internal: int) -> list:
        out = (C.c_size_t * self.sub_chunk_no)()
        n = C.c_size_t()
        err = OcError()
        if lib().oc_repair_subchunk_indices(C.byref(self._c), lost_internal, out, C.byref(n),
                                            C.byref(err)):
            raise OracleError(err)
        return [int(out[i]) for i in range(n.value)]

    def normalized_repair_bandwidth(self) -> float:
        return float(lib().oc_normalized_repair_bandwidth(C.byref(self._c)))

    def encoded_chunk_size(self, data_len: int) -> int:
        return int(lib().oc_encoded_chunk_size(C.byref(self._c), data_len))

    def encode_array(self, data: np.ndarray) -> np.ndarray:
        """Returns an (n, chunk_size) uint8 array: k data chunks then m parity."""
        data = _as_np(data)
        chunk = self.encoded_chunk_size(data.size)
        out = np.zeros((self.n, chunk), dtype=np.uint8)
        err = OcError()
        if lib().oc_encode(C.byref(self._c), _u8(data) if data.size else None, data.size,
                           _u8(out), C.byref(err)):
            raise OracleError(err)
        return out

    def encode(self, data) -> list:
        return [bytes(r) for r in self.encode_array(data)]

    def decode(self, available: dict, erasures) -> bytes:
        ids = list(available.keys())
        arrs = [_as_np(available[i]) for i in ids]
        ptrs = (C.POINTER(C.c_uint8) * max(1, len(arrs)))(*[_u8(a) for a in arrs])
        lens = _sizes([a.size for a in arrs])
        er = _sizes(list(erasures))
        cap = self.k * (arrs[0].size if arrs else 0)
        out = np.zeros(max(cap, 1), dtype=np.uint8)
        olen = C.c_size_t()
        err = OcError()
        if lib().oc_decode(C.byref(self._c), _sizes(ids), ptrs, lens, len(ids), er,
                           len(list(erasures)), _u8(out), cap, C.byref(olen), C.byref(err)):
            raise OracleError(err)
        return out[:olen.value].tobytes()

    def minimum_to_repair(self, lost: int, available) -> list:
        av = list(available)
        helpers = (C.c_size_t * max(1, self.d))()
        idx = (C.c_size_t * self.sub_chunk_no)()
        nh, ni = C.c_size_t(), C.c_size_t()
        err = OcError()
        if lib().oc_minimum_to_repair(C.byref(self._c), lost, _sizes(av), len(av), helpers,
                                      C.byref(nh), idx, C.byref(ni), C.byref(err)):
            raise OracleError(err)
        il = [int(idx[i]) for i in range(ni.value)]
        return [(int(helpers[i]), list(il)) for i in range(nh.value)]

    def repair(self, lost: int, helper_data: dict, chunk_size: int) -> bytes:
        ids = list(helper_data.keys())
        arrs = [_as_np(helper_data[i]) for i in ids]
        ptrs = (C.POINTER(C.c_uint8) * max(1, len(arrs)))(*[_u8(a) for a in arrs])
        out = np.zeros(max(chunk_size, 1), dtype=np.uint8)
        err = OcError()
        if lib().oc_repair(C.byref(self._c), lost, _sizes(ids), ptrs,
                           _sizes([a.size for a in arrs]), len(ids), chunk_size, _u8(out),
                           C.byref(err)):
            raise OracleError(err)
        return out[:chunk_size].tobytes()

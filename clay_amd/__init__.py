"""clay_amd -- MI355X-native Clay (Coupled-Layer MSR) erasure codes.

Python mirror of the reference's public API, `clay_codes::ClayCode`
(spool-labs/clay, src/lib.rs:57-242), over the C ABI in include/clay.h.  Same
names, same argument meaning, same error variants (src/error.rs:5-24) raised as
`ClayError` subclasses.  All byte work runs in HIP kernels on the GPU
(libclay_amd.so); there is no CPU fallback.

    >>> from clay_amd import ClayCode
    >>> clay = ClayCode(4, 2, 5)
    >>> chunks = clay.encode(b"Hello, Clay codes!")
    >>> avail = {i: c for i, c in enumerate(chunks) if i != 0}
    >>> clay.decode(avail, [0])[:18]
    b'Hello, Clay codes!'
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import ClayCodeStruct, ClayErrorStruct

__all__ = [
    "ClayCode", "ClayError", "InvalidParameters", "InsufficientHelpers", "InvalidChunkSize",
    "InsufficientHelperData", "InconsistentChunkSizes", "TooManyErasures",
    "ReconstructionFailed", "MissingYSectionHelper", "Overflow", "DeviceError",
    "set_encode_path", "last_encode_path", "last_launch_count", "set_exec_mode", "last_exec_path",
]


class ClayError(Exception):
    """ClayError (error.rs:5-24).  `fields` holds the variant payload in
    declaration order; str(e) is the reference Display text (error.rs:26-54)."""
    kind = 0
    name = "ClayError"

    def __init__(self, msg: str, fields: Tuple[int, int, int] = (0, 0, 0)):
        super().__init__(msg)
        self.msg = msg
        self.fields = fields


class InvalidParameters(ClayError): kind, name = 1, "InvalidParameters"
class InsufficientHelpers(ClayError): kind, name = 2, "InsufficientHelpers"
class InvalidChunkSize(ClayError): kind, name = 3, "InvalidChunkSize"
class InsufficientHelperData(ClayError): kind, name = 4, "InsufficientHelperData"
class InconsistentChunkSizes(ClayError): kind, name = 5, "InconsistentChunkSizes"
class TooManyErasures(ClayError): kind, name = 6, "TooManyErasures"
class ReconstructionFailed(ClayError): kind, name = 7, "ReconstructionFailed"
class MissingYSectionHelper(ClayError): kind, name = 8, "MissingYSectionHelper"
class Overflow(ClayError): kind, name = 9, "Overflow"
class DeviceError(ClayError): kind, name = 100, "DeviceError"


_BY_KIND = {c.kind: c for c in (InvalidParameters, InsufficientHelpers, InvalidChunkSize,
                                InsufficientHelperData, InconsistentChunkSizes, TooManyErasures,
                                ReconstructionFailed, MissingYSectionHelper, Overflow,
                                DeviceError)}


def _raise(rc: int, err: ClayErrorStruct):
    cls = _BY_KIND.get(int(err.kind) or rc, ClayError)
    raise cls(err.msg.decode(errors="replace"), (int(err.a), int(err.b), int(err.c)))


def _u8(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def _np(b) -> np.ndarray:
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b.reshape(-1), dtype=np.uint8)
    return np.frombuffer(memoryview(b).cast("B"), dtype=np.uint8) if len(b) else np.zeros(0, np.uint8)


def _sizes(vals) -> "C.Array":
    vals = [int(v) for v in vals]
    return (C.c_size_t * max(1, len(vals)))(*vals)


def _ptr(x) -> int:
    """Address of a torch tensor, a numpy array or a raw int."""
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    if hasattr(x, "__array_interface__"):
        return int(x.__array_interface__["data"][0])
    return int(x)


_ENCODE_PATHS = {"auto": 0, "staged": 1, "fused": 2, "bitsliced": 3, "stream": 5}


def set_encode_path(mode: str, tile: int = 0) -> str:
    """Process-wide encode path: 'auto' | 'staged' | 'fused' | 'bitsliced' | 'stream'.

    `tile` selects a variant: 'bitsliced' lanes per column group (0, 1, 4), 'stream' loader
    waves for (10,4,13) (0 = default 4, 1, 2, 4; (9,4,12) always runs 4; (9,3,11) 2, or 7 for
    variant 7). 'stream' (10,4,13) / (9,4,12) needs 8-byte rows (sc % 8 == 0).
    Every accepted path produces the reference's parity; anything else raises ValueError.
    Returns the previous path name."""
    if mode not in _ENCODE_PATHS:
        raise ValueError(f"unknown encode path {mode!r}")
    prev = _lib.lib().clay_set_encode_path(_ENCODE_PATHS[mode] | (int(tile) << 8))
    if prev < 0:
        raise ValueError(f"encode path {mode!r} has no variant {tile}")
    return {v: k for k, v in _ENCODE_PATHS.items()}.get(prev & 0xFF, "auto")


_EXEC_MODES = {"auto": 0, "grouped": 1, "tile": 2, "stream": 3, "stream-local": 5, "stream-fused2": 6}


def set_exec_mode(mode: str) -> str:
    """Process-wide plan executor for decode / repair / staged encode (clay.h): 'auto' (tile-fused
    where the U slots fit in LDS, else grouped; for q = 4, t = 4 codes the local decode for
    erasures in one y-section plus at most one other, the fused decode v2 for 3-4 erasures in
    distinct y-sections; the bit-sliced repair kernels for q = m repairs from all n - 1 nodes),
    'grouped' (one launch per level), 'tile', 'stream' (every decode a streaming kernel takes:
    local, else fused v2 from 2 erasures; the streaming repair kernel at any sub-chunk size),
    'stream-local' or 'stream-fused2' (that kernel wherever it applies).  Modes choose kernels
    only: every mode returns the reference's bytes on any input.  Returns the previous mode."""
    if mode not in _EXEC_MODES:
        raise ValueError(f"unknown exec mode {mode!r}")
    prev = _lib.lib().clay_set_exec_mode(_EXEC_MODES[mode])
    return {v: k for k, v in _EXEC_MODES.items()}[prev]


def last_exec_path() -> str:
    """Plan executor of this thread's last decode / repair / staged encode: 'tile' | 'grouped' |
    'stream-local256' | 'stream-local' | 'stream-fused2' | 'bs-repair-stream' | 'bs-repair' | 'none'."""
    return _lib.lib().clay_last_exec_path().decode()


def release_workspace(device: int = 0) -> None:
    """Free the device's idle pooled buffers and batch pointer tables (clay.h)."""
    err = ClayErrorStruct()
    rc = _lib.lib().clay_release_workspace(int(device), C.byref(err))
    if rc:
        _raise(rc, err)


def release_captured(device: int = 0) -> None:
    """Reclaim the pointer-table arena and the pooled workspaces that calls inside stream
    captures left to their graphs; call once every replay of those graphs has completed and the
    graphs are destroyed (clay.h: no device-wide synchronize is taken)."""
    err = ClayErrorStruct()
    rc = _lib.lib().clay_release_captured(int(device), C.byref(err))
    if rc:
        _raise(rc, err)


def workspace_bytes(device: int = 0) -> int:
    """Device memory held by the device's buffer pool."""
    return int(_lib.lib().clay_workspace_bytes(int(device)))


def last_encode_path() -> str:
    return _lib.lib().clay_last_encode_path().decode()


def last_launch_count() -> int:
    return int(_lib.lib().clay_last_launch_count())


class ClayCode:
    """Clay (Coupled-Layer) erasure code (lib.rs:57-82).

    Fields k, m, n, d, q, t, nu, sub_chunk_no, beta as in the reference."""

    def __init__(self, k: int, m: int, d: int):
        self._c = ClayCodeStruct()
        err = ClayErrorStruct()
        rc = _lib.lib().clay_new(int(k), int(m), int(d), C.byref(self._c), C.byref(err))
        if rc:
            _raise(rc, err)
        for name, _ in ClayCodeStruct._fields_:
            if name not in ("original_count", "recovery_count"):
                setattr(self, name, int(getattr(self._c, name)))

    # lib.rs:94 / :150
    @classmethod
    def new(cls, k: int, m: int, d: int) -> "ClayCode":
        return cls(k, m, d)

    @classmethod
    def new_default(cls, k: int, m: int) -> "ClayCode":
        return cls(k, m, k + m - 1)

    def __repr__(self):
        return (f"ClayCode {{ k: {self.k}, m: {self.m}, n: {self.n}, d: {self.d}, q: {self.q}, "
                f"t: {self.t}, nu: {self.nu}, sub_chunk_no: {self.sub_chunk_no}, "
                f"beta: {self.beta} }}")

    def clone(self) -> "ClayCode":
        return ClayCode(self.k, self.m, self.d)

    @property
    def struct(self) -> ClayCodeStruct:
        return self._c

    # lib.rs:239-241
    def normalized_repair_bandwidth(self) -> float:
        return float(_lib.lib().clay_normalized_repair_bandwidth(C.byref(self._c)))

    def encoded_chunk_size(self, data_len: int) -> int:
        return int(_lib.lib().clay_encoded_chunk_size(C.byref(self._c), int(data_len)))

    # lib.rs:176-178
    def encode_array(self, data) -> np.ndarray:
        """encode() into one (n, chunk_size) uint8 array (k data rows, then m parity)."""
        arr = _np(data)
        chunk = self.encoded_chunk_size(arr.size)
        out = np.empty((self.n, chunk), dtype=np.uint8)
        ptrs = (C.POINTER(C.c_uint8) * self.n)(*[_u8(out[i]) for i in range(self.n)])
        err = ClayErrorStruct()
        rc = _lib.lib().clay_encode(C.byref(self._c), _u8(arr) if arr.size else None, arr.size,
                                    ptrs, chunk, C.byref(err))
        if rc:
            _raise(rc, err)
        return out

    def encode(self, data) -> List[bytes]:
        return [bytes(r) for r in self.encode_array(data)]

    # lib.rs:188-194
    def decode(self, available: Dict[int, bytes], erasures: Sequence[int]) -> bytes:
        ids = list(available.keys())
        arrs = [_np(available[i]) for i in ids]
        ptrs = (C.POINTER(C.c_uint8) * max(1, len(arrs)))(*[_u8(a) for a in arrs])
        lens = _sizes([a.size for a in arrs])
        er = list(erasures)
        cap = self.k * (arrs[0].size if arrs else 0)
        out = np.empty(max(cap, 1), dtype=np.uint8)
        olen = C.c_size_t()
        err = ClayErrorStruct()
        rc = _lib.lib().clay_decode(C.byref(self._c), _sizes(ids), ptrs, lens, len(ids), _sizes(er),
                                    len(er), _u8(out), cap, C.byref(olen), C.byref(err))
        if rc:
            _raise(rc, err)
        return out[:olen.value].tobytes()

    # lib.rs:207-213
    def minimum_to_repair(self, lost_node: int, available: Sequence[int]) -> List[Tuple[int, List[int]]]:
        av = list(available)
        helpers = (C.c_size_t * max(1, self.d))()
        sub = (C.c_size_t * max(1, self.sub_chunk_no))()
        nh, ns = C.c_size_t(), C.c_size_t()
        err = ClayErrorStruct()
        rc = _lib.lib().clay_minimum_to_repair(C.byref(self._c), int(lost_node), _sizes(av), len(av),
                                               helpers, C.byref(nh), sub, C.byref(ns), C.byref(err))
        if rc:
            _raise(rc, err)
        idx = [int(sub[i]) for i in range(ns.value)]
        return [(int(helpers[i]), list(idx)) for i in range(nh.value)]

    # lib.rs:226-233
    def repair(self, lost_node: int, helper_data: Dict[int, bytes], chunk_size: int) -> bytes:
        ids = list(helper_data.keys())
        arrs = [_np(helper_data[i]) for i in ids]
        ptrs = (C.POINTER(C.c_uint8) * max(1, len(arrs)))(*[_u8(a) for a in arrs])
        out = np.empty(max(int(chunk_size), 1), dtype=np.uint8)
        err = ClayErrorStruct()
        rc = _lib.lib().clay_repair(C.byref(self._c), int(lost_node), _sizes(ids), ptrs,
                                    _sizes([a.size for a in arrs]), len(ids), int(chunk_size),
                                    _u8(out), C.byref(err))
        if rc:
            _raise(rc, err)
        return out[:int(chunk_size)].tobytes()

    # ---- device-resident API (HBM in / HBM out) ------------------------------
    def encode_device(self, data_chunks, parity_chunks, chunk_size: int, device: int = 0,
                      stream: int = 0):
        """data_chunks: k device buffers (torch tensors or pointers), parity_chunks: m."""
        dp = (C.c_void_p * self.k)(*[_ptr(x) for x in data_chunks])
        pp = (C.c_void_p * self.m)(*[_ptr(x) for x in parity_chunks])
        err = ClayErrorStruct()
        rc = _lib.lib().clay_encode_device(C.byref(self._c), dp, pp, int(chunk_size), int(device),
                                           C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

    def encode_device_batch(self, data_chunks, parity_chunks, n_stripes: int, chunk_size: int,
                            device: int = 0, stream: int = 0):
        dp = (C.c_void_p * (self.k * n_stripes))(*[_ptr(x) for x in data_chunks])
        pp = (C.c_void_p * (self.m * n_stripes))(*[_ptr(x) for x in parity_chunks])
        err = ClayErrorStruct()
        rc = _lib.lib().clay_encode_device_batch(C.byref(self._c), dp, pp, int(n_stripes),
                                                 int(chunk_size), int(device),
                                                 C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

    def encode_device_strided(self, data, parity, n_stripes: int, chunk_size: int, data_node_stride: int = 0,
                              data_stripe_stride: int = 0, parity_node_stride: int = 0,
                              parity_stripe_stride: int = 0, device: int = 0, stream: int = 0):
        """Batched encode of stripes at fixed strides (clay.h clay_encode_device_strided).
        Strides default to a contiguous [n_stripes][k or m][chunk_size] layout."""
        dns = data_node_stride or chunk_size
        dss = data_stripe_stride or self.k * chunk_size
        pns = parity_node_stride or chunk_size
        pss = parity_stripe_stride or self.m * chunk_size
        err = ClayErrorStruct()
        rc = _lib.lib().clay_encode_device_strided(C.byref(self._c), C.c_void_p(_ptr(data)), dns, dss,
                                                   C.c_void_p(_ptr(parity)), pns, pss, int(n_stripes),
                                                   int(chunk_size), int(device), C.c_void_p(int(stream)),
                                                   C.byref(err))
        if rc:
            _raise(rc, err)

    def chunk_to_ygroup(self, y: int, chunk, group, chunk_size: int, device: int = 0, stream: int = 0):
        """Reorder a device chunk into the y-grouped layout of y-section y (clay.h)."""
        err = ClayErrorStruct()
        rc = _lib.lib().clay_chunk_to_ygroup(C.byref(self._c), int(y), C.c_void_p(_ptr(chunk)),
                                             C.c_void_p(_ptr(group)), int(chunk_size), int(device),
                                             C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

    def ygroup_to_chunk(self, y: int, group, chunk, chunk_size: int, device: int = 0, stream: int = 0):
        """Inverse of chunk_to_ygroup."""
        err = ClayErrorStruct()
        rc = _lib.lib().clay_ygroup_to_chunk(C.byref(self._c), int(y), C.c_void_p(_ptr(group)),
                                             C.c_void_p(_ptr(chunk)), int(chunk_size), int(device),
                                             C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

    def reserve_workspace(self, chunk_size: int, device: int = 0):
        """Pre-allocate a pooled workspace and upload the encode plan (clay.h)."""
        err = ClayErrorStruct()
        rc = _lib.lib().clay_reserve_workspace(C.byref(self._c), int(chunk_size), int(device), C.byref(err))
        if rc:
            _raise(rc, err)

    def encode_host_pipelined(self, data_chunks, parity_chunks, chunk_size: int, device: int = 0,
                              piece_bytes: int = 0, n_streams: int = 0):
        """Host-streaming encode (clay.h clay_encode_host_pipelined): k host data buffers in,
        m host parity buffers out (numpy arrays or CPU tensors; pinned tensors overlap H2D,
        encode and D2H).  Blocks until the parity is in host memory."""
        dp = (C.c_void_p * self.k)(*[_ptr(x) for x in data_chunks])
        pp = (C.c_void_p * self.m)(*[_ptr(x) for x in parity_chunks])
        err = ClayErrorStruct()
        rc = _lib.lib().clay_encode_host_pipelined(C.byref(self._c), dp, pp, int(chunk_size),
                                                   int(device), int(piece_bytes), int(n_streams),
                                                   C.byref(err))
        if rc:
            _raise(rc, err)

    def decode_device(self, chunks, erasures: Sequence[int], out_chunks, chunk_size: int,
                      device: int = 0, stream: int = 0, codeword: bool = False):
        """chunks / out_chunks: n entries, None where absent (see clay.h).  codeword=True calls
        clay_decode_device_codeword: the caller vouches that the chunks are one codeword, so a
        single erasure may be rebuilt by the repair kernel (1/q of every chunk read); for this
        call only."""
        cp = (C.c_void_p * self.n)(*[(_ptr(x) if x is not None else None) for x in chunks])
        op = (C.c_void_p * self.n)(*[(_ptr(x) if x is not None else None) for x in out_chunks])
        er = list(erasures)
        err = ClayErrorStruct()
        fn = _lib.lib().clay_decode_device_codeword if codeword else _lib.lib().clay_decode_device
        rc = fn(C.byref(self._c), cp, _sizes(er), len(er), op, int(chunk_size), int(device),
                C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

    def repair_device_full_chunks(self, lost_node: int, helper_ids: Sequence[int], helper_chunks,
                                  chunk_size: int, out, device: int = 0, stream: int = 0):
        """Repair from whole helper chunks resident on the device (clay.h
        clay_repair_device_full_chunks): no gather of the beta repair layers."""
        ids = list(helper_ids)
        hp = (C.c_void_p * max(1, len(ids)))(*[_ptr(x) for x in helper_chunks])
        err = ClayErrorStruct()
        rc = _lib.lib().clay_repair_device_full_chunks(C.byref(self._c), int(lost_node), _sizes(ids),
                                                       hp, len(ids), int(chunk_size),
                                                       C.c_void_p(_ptr(out)), int(device),
                                                       C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

    def repair_device(self, lost_node: int, helper_ids: Sequence[int], helper_bufs, chunk_size: int,
                      out, device: int = 0, stream: int = 0):
        ids = list(helper_ids)
        hp = (C.c_void_p * max(1, len(ids)))(*[_ptr(x) for x in helper_bufs])
        err = ClayErrorStruct()
        rc = _lib.lib().clay_repair_device(C.byref(self._c), int(lost_node), _sizes(ids), hp,
                                           len(ids), int(chunk_size), C.c_void_p(_ptr(out)),
                                           int(device), C.c_void_p(int(stream)), C.byref(err))
        if rc:
            _raise(rc, err)

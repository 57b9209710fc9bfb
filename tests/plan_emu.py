"""TEST INFRASTRUCTURE: execute an exported staged-engine plan (clay_plan_export)
on the CPU with numpy, to check the host planner against the oracle without a GPU.
This is a checker for the planner only; the product executes plans in HIP."""
from __future__ import annotations

import ctypes as C

import numpy as np

from clay_amd import _lib, _raise
from clay_amd._lib import ClayErrorStruct

_MUL = None


def mul_table() -> np.ndarray:
    global _MUL
    if _MUL is None:
        exp = np.zeros(512, np.int64)
        log = np.zeros(256, np.int64)
        b = 1
        for i in range(255):
            exp[i] = b
            log[b] = i
            b <<= 1
            if b & 0x100:
                b ^= 0x11D
        exp[255:510] = exp[:255]
        t = np.zeros((256, 256), np.uint8)
        a = np.arange(1, 256)
        t[1:, 1:] = exp[(log[a][:, None] + log[a][None, :])].astype(np.uint8)
        _MUL = t
    return _MUL


def export_plan(code, kind: int, mask=None, want=None, lost: int = 0):
    L = _lib.lib()
    tn = code.q * code.t
    m = (C.c_uint8 * tn)(*(mask if mask is not None else [0] * tn))
    w = (C.c_uint8 * tn)(*(want if want is not None else [0] * tn))
    counts = (C.c_size_t * 3)()
    err = ClayErrorStruct()
    rc = L.clay_plan_export(C.byref(code.struct), kind, m, w, lost, None, 0, None, 0, None, 0, counts,
                            C.byref(err))
    if rc:
        _raise(rc, err)
    ops = np.zeros(counts[0] * 4 + 4, np.uint32)
    srcs = np.zeros(counts[1] * 4 + 4, np.uint32)
    stages = np.zeros(counts[2] + 1, np.uint32)
    P = C.POINTER(C.c_uint32)
    rc = L.clay_plan_export(C.byref(code.struct), kind, m, w, lost,
                            ops.ctypes.data_as(P), ops.size, srcs.ctypes.data_as(P), srcs.size,
                            stages.ctypes.data_as(P), stages.size, counts, C.byref(err))
    if rc:
        _raise(rc, err)
    return (ops[:counts[0] * 4].reshape(-1, 4), srcs[:counts[1] * 4].reshape(-1, 4),
            stages[:counts[2]])


def run_plan(code, plan, bufs: dict, sc: int):
    """bufs: base index -> (nslots, sc) uint8 arrays (C/H/U/OUT)."""
    ops, srcs, stages = plan
    T = mul_table()
    for s in range(len(stages) - 1):
        results = []
        for i in range(stages[s], stages[s + 1]):
            base, slot, sb, ns = (int(v) for v in ops[i])
            acc = np.zeros(sc, np.uint8)
            for j in range(sb, sb + ns):
                b, sl, coef = int(srcs[j][0]), int(srcs[j][1]), int(srcs[j][2])
                acc ^= T[coef][bufs[b][sl]]
            results.append((base, slot, acc))
        for base, slot, acc in results:  # stage = one launch: all reads before writes
            bufs[base][slot] = acc
    return bufs

#!/usr/bin/env python3
"""Host-inclusive rates of the drop-in host-buffer API (clay_encode / clay_decode /
clay_repair: host memory in, host memory out, PCIe both ways; the north-star path starts
and ends in host memory).  Pinned (hipHostMalloc via torch pin_memory) and pageable
(numpy) buffers; BASELINE configs: (10,4,13) 1 GiB encode and 4-erasure decode,
(9,3,11) repair of node 0 at chunk 268,435,458.  One JSON object per line.

rate = user payload bytes / wall time: the stripe for encode, the k returned data chunks
for decode, the rebuilt chunk for repair; `pcie_bytes` is what crosses the link."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clay_amd import ClayCode, _lib  # noqa: E402
from clay_amd._lib import ClayErrorStruct  # noqa: E402

L = _lib.lib()
REPS = int(os.environ.get("REPS", "5"))
U8P = C.POINTER(C.c_uint8)


def buf(n, pinned):
    if pinned:
        return torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
    return np.empty(n, np.uint8)


def p8(a):
    return a.ctypes.data_as(U8P)


def sizes(v):
    return (C.c_size_t * max(1, len(v)))(*v)


def timed(fn):
    fn()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def check(rc, err):
    if rc:
        raise RuntimeError(err.msg.decode())


def encode(pinned):
    c = ClayCode(10, 4, 13)
    n = 1 << 30
    chunk = c.encoded_chunk_size(n)
    data = buf(n, pinned)
    data[:] = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8)
    outs = [buf(chunk, pinned) for _ in range(14)]
    optr = (U8P * 14)(*[p8(o) for o in outs])
    err = ClayErrorStruct()
    t = timed(lambda: check(L.clay_encode(C.byref(c.struct), p8(data), n, optr, chunk, C.byref(err)), err))
    return {"op": "clay_encode (10,4,13) 1 GiB", "pinned": pinned, "ms": round(t * 1e3, 2),
            "GiBps": round(n / t / 2**30, 2), "pcie_bytes": 14 * chunk}, (c, outs, chunk)


def decode(pinned, enc):
    c, outs, chunk = enc
    er = [0, 4, 8, 12]
    ids = [i for i in range(14) if i not in er]
    src = [outs[i] if pinned else np.array(outs[i]) for i in ids]
    bp = (U8P * len(ids))(*[p8(b) for b in src])
    out = buf(10 * chunk, pinned)
    olen = C.c_size_t()
    err = ClayErrorStruct()
    t = timed(lambda: check(L.clay_decode(C.byref(c.struct), sizes(ids), bp, sizes([chunk] * len(ids)), len(ids),
                                          sizes(er), len(er), p8(out), out.size, C.byref(olen), C.byref(err)), err))
    assert np.array_equal(out[:chunk], outs[0]) and np.array_equal(out[8 * chunk:9 * chunk], outs[8])
    return {"op": "clay_decode (10,4,13) 1 GiB, erasures [0,4,8,12]", "pinned": pinned, "ms": round(t * 1e3, 2),
            "GiBps": round(10 * chunk / t / 2**30, 2), "pcie_bytes": 10 * chunk + 3 * chunk}


def repair(pinned):
    c = ClayCode(9, 3, 11)
    chunk = 268_435_458
    sc = chunk // c.sub_chunk_no
    info = c.minimum_to_repair(0, list(range(1, 12)))
    ids = [h for h, _ in info]
    hb = [buf(27 * sc, pinned) for _ in ids]
    rng = np.random.default_rng(2)
    for b in hb:
        b[:] = rng.integers(0, 256, b.size, dtype=np.uint8)
    bp = (U8P * len(ids))(*[p8(b) for b in hb])
    out = buf(chunk, pinned)
    err = ClayErrorStruct()
    t = timed(lambda: check(L.clay_repair(C.byref(c.struct), 0, sizes(ids), bp, sizes([27 * sc] * len(ids)),
                                          len(ids), chunk, p8(out), C.byref(err)), err))
    return {"op": "clay_repair (9,3,11) node 0, chunk 268435458", "pinned": pinned, "ms": round(t * 1e3, 2),
            "GiBps": round(chunk / t / 2**30, 2), "pcie_bytes": 11 * 27 * sc + chunk}


if __name__ == "__main__":
    for pinned in (True, False):
        r, enc = encode(pinned)
        print(json.dumps(r), flush=True)
        print(json.dumps(decode(pinned, enc)), flush=True)
        del enc
        print(json.dumps(repair(pinned)), flush=True)

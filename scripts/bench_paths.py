#!/usr/bin/env python3
"""Device-resident timing of every SURVEY.md §8 configuration on one GPU (inputs resident in
HBM, HIP events on the launch stream, median of N runs).  Algorithmic bytes per SURVEY §8(d):
encode  read k*chunk + write m*chunk
decode  read (n-e)*chunk + write (#erased data nodes)*chunk
repair  read d*beta*sc + write chunk
Prints one JSON object per configuration."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import clay_amd  # noqa: E402
from clay_amd import ClayCode  # noqa: E402

RUNS = int(os.environ.get("RUNS", "10"))
EXEC = os.environ.get("CLAY_EXEC", "auto")  # exec mode: auto | grouped | tile | stream | stream-local | stream-fused2
clay_amd.set_exec_mode(EXEC)
stream = torch.cuda.current_stream()


B2B = int(os.environ.get("B2B", "8"))  # back-to-back calls per timed sample


def timed(fn):
    """Median / min per-call time of B2B back-to-back calls between two events: the host work of
    call i+1 (argument marshalling, validation, launch) overlaps the kernel of call i, so the
    sample is device time, not Python overhead (one call on an idle GPU would time both)."""
    ts = []
    for i in range(RUNS + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()  # queue one call ahead so e0 is recorded behind work, not on an idle GPU
        e0.record(stream)
        for _ in range(B2B):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1) / B2B)
    return float(np.median(ts)), float(np.min(ts))


def report(name, ms, mn, algo, extra=None):
    d = {"config": name, "median_ms": round(ms, 4), "min_ms": round(mn, 4),
         "algorithmic_bytes": int(algo), "GBps": round(algo / (ms * 1e-3) / 1e9, 1),
         "frac_of_8TBps": round(algo / (ms * 1e-3) / 8e12, 4), "path": (clay_amd.last_encode_path() if name.startswith("encode")
                  else clay_amd.last_exec_path()),
         "launches": clay_amd.last_launch_count()}
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)


def rnd(n, chunk, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    return torch.randint(0, 256, (n, chunk), dtype=torch.uint8, device="cuda", generator=g)


def encode_cfg(k, m, d, stripe, path=None):
    if path:
        clay_amd.set_encode_path(path, 0)
    try:
        _encode_cfg(k, m, d, stripe)
    finally:
        if path:
            clay_amd.set_encode_path("auto", 0)


def _encode_cfg(k, m, d, stripe):
    c = ClayCode(k, m, d)
    chunk = c.encoded_chunk_size(stripe)
    data, par = rnd(k, chunk, 1), torch.empty((m, chunk), dtype=torch.uint8, device="cuda")
    ms, mn = timed(lambda: c.encode_device([data[i] for i in range(k)], [par[i] for i in range(m)], chunk, 0,
                                           stream.cuda_stream))
    report(f"encode ({k},{m},{d}) {stripe >> 20} MiB", ms, mn, (k + m) * chunk)


def encode_batch_cfg(k, m, d, stripe, n):
    """clay_bench.rs shape (1 MiB stripes) as one device batch call: n stripes per call."""
    c = ClayCode(k, m, d)
    chunk = c.encoded_chunk_size(stripe)
    data, par = rnd(n * k, chunk, 5), torch.empty((n * m, chunk), dtype=torch.uint8, device="cuda")
    dl, pl = [data[i] for i in range(n * k)], [par[i] for i in range(n * m)]
    ms, mn = timed(lambda: c.encode_device_batch(dl, pl, n, chunk, 0, stream.cuda_stream))
    report(f"encode ({k},{m},{d}) batch {n} x {stripe >> 10} KiB", ms, mn, n * (k + m) * chunk,
           {"input_GiBps": round(n * k * chunk / (ms * 1e-3) / 2**30, 1)})


def decode_cfg(k, m, d, stripe, er, mode=None, codeword=False):
    prev = clay_amd.set_exec_mode(mode) if mode else None
    try:
        _decode_cfg(k, m, d, stripe, er, codeword)
    finally:
        if prev:
            clay_amd.set_exec_mode(prev)


def _decode_cfg(k, m, d, stripe, er, codeword=False):
    c = ClayCode(k, m, d)
    chunk = c.encoded_chunk_size(stripe)
    full = rnd(c.n, chunk, 2)
    outs = torch.empty((c.n, chunk), dtype=torch.uint8, device="cuda")
    ins = [None if i in er else full[i] for i in range(c.n)]
    ous = [outs[i] if i in er else None for i in range(c.n)]
    ms, mn = timed(lambda: c.decode_device(ins, er, ous, chunk, 0, stream.cuda_stream, codeword=codeword))
    ndata = sum(1 for e in er if e < k)
    name = f"decode ({k},{m},{d}) {stripe >> 20} MiB erasures {er}"
    if codeword and clay_amd.last_exec_path() == "bs-repair-stream":
        # the repair route reads the beta = alpha / q layers of every other chunk and writes the
        # erased chunk: charged the bytes it moves (a decode's full-read bytes would put frac > 1)
        beta_bytes = chunk // c.q
        report(name + " codeword", ms, mn, (c.n - 1) * beta_bytes + chunk,
               {"bytes_counted": "repair route: (n-1) x chunk/q read + the erased chunk written"})
    else:
        report(name + (" codeword" if codeword else ""), ms, mn, (c.n - len(er)) * chunk + ndata * chunk,
               {"writes_counted": "erased data nodes only"})


def repair_cfg(k, m, d, chunk, lost):
    c = ClayCode(k, m, d)
    sc = chunk // c.sub_chunk_no
    info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
    helpers = [h for h, _ in info]
    beta = len(info[0][1])
    hb = rnd(len(helpers), beta * sc, 3)
    out = torch.empty(chunk, dtype=torch.uint8, device="cuda")
    ms, mn = timed(lambda: c.repair_device(lost, helpers, [hb[i] for i in range(len(helpers))], chunk, out, 0,
                                           stream.cuda_stream))
    report(f"repair ({k},{m},{d}) chunk {chunk} node {lost}", ms, mn, len(helpers) * beta * sc + chunk)
    del hb
    # same repair straight from whole helper chunks in HBM (only the beta layers are read)
    full = rnd(len(helpers), chunk, 4)
    ms, mn = timed(lambda: c.repair_device_full_chunks(lost, helpers, [full[i] for i in range(len(helpers))],
                                                       chunk, out, 0, stream.cuda_stream))
    report(f"repair ({k},{m},{d}) chunk {chunk} node {lost} from full chunks", ms, mn,
           len(helpers) * beta * sc + chunk)


def prewarm(ms=250.0):
    """Untimed load so every configuration is timed at the GPU's sustained clock."""
    import time
    c = ClayCode(10, 4, 13)
    chunk = c.encoded_chunk_size(1 << 30)
    data, par = rnd(10, chunk, 9), torch.empty((4, chunk), dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            c.encode_device([data[i] for i in range(10)], [par[i] for i in range(4)], chunk, 0, stream.cuda_stream)
        torch.cuda.synchronize()


if __name__ == "__main__":
    prewarm(float(os.environ.get("PREWARM_MS", "250")))
    only = os.environ.get("ONLY", "encode,batch,decode,repair").split(",")
    jobs = [("encode", lambda: encode_cfg(10, 4, 13, 1 << 30)),
            ("encode", lambda: encode_cfg(4, 2, 5, 64 << 20)),
            ("encode", lambda: encode_cfg(9, 3, 11, 9 * (256 << 20))),
            ("batch", lambda: encode_batch_cfg(4, 2, 5, 1 << 20, 256)),
            ("decode", lambda: decode_cfg(4, 2, 5, 64 << 20, [0])),
            ("decode", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8, 12])),
            ("decode", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8, 12], "grouped")),
            ("cfg5", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8, 12])),  # under CLAY_EXEC
            ("c2e", lambda: encode_cfg(4, 2, 5, 64 << 20)),
            ("c2e", lambda: encode_cfg(4, 2, 5, 64 << 20, "bitsliced")),
            ("cfg2", lambda: decode_cfg(4, 2, 5, 64 << 20, [0])),  # under CLAY_EXEC
            ("cfg2", lambda: decode_cfg(4, 2, 5, 64 << 20, [5])),
            # the fused decode v2 for 3 and 2 erasures in distinct sections (auto: split / local)
            ("f2x", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8], "stream-fused2")),
            ("f2x", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8])),
            ("f2x", lambda: decode_cfg(10, 4, 13, 1 << 30, [1, 9, 13], "stream-fused2")),
            ("f2x", lambda: decode_cfg(10, 4, 13, 1 << 30, [1, 9, 13])),
            ("f2x", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4], "stream-fused2")),
            ("f2x", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4])),
            ("decode", lambda: decode_cfg(10, 4, 13, 1 << 30, [0])),
            ("decode23", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4])),
            ("decode23", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4, 8])),
            # same-section and mixed patterns (the local decode in auto)
            ("decodeL", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1])),
            ("decodeL", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 4])),
            ("decodeL", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 2, 3])),
            ("decodeL", lambda: decode_cfg(10, 4, 13, 1 << 30, [12])),
            # the local decodes: 256-byte row runs ({0}, {12}, {0,4}) and 64-byte tiles ({0,1})
            ("local", lambda: decode_cfg(10, 4, 13, 1 << 30, [0])),
            ("local", lambda: decode_cfg(10, 4, 13, 1 << 30, [12])),
            ("local", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 4])),
            ("local", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1])),
            ("local", lambda: decode_cfg(9, 4, 12, 1 << 30, [0])),
            ("local", lambda: decode_cfg(9, 4, 12, 1 << 30, [0, 4])),
            # round 6: 4-erasure patterns with two erasures in one section ((2,1,1) and (2,2)
            # sections: 750 of the 1,001 4-erasure patterns), k_stream_fused2 in auto, and the
            # grouped executor they ran on before; {0,8,9,10} runs a split step (neighbouring
            # sections beyond the ring)
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 4, 8])),
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 4, 12])),
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 4, 5])),
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [8, 9, 0, 4])),
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 8, 9, 10])),
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 4, 8], "grouped")),
            ("two", lambda: decode_cfg(10, 4, 13, 1 << 30, [0, 1, 4, 5], "grouped")),
            # clay_decode_device_codeword: one erasure rebuilt by the repair kernel from whole
            # chunks (charged the repair route's bytes)
            ("codeword", lambda: decode_cfg(10, 4, 13, 1 << 30, [0], codeword=True)),
            ("codeword", lambda: decode_cfg(10, 4, 13, 1 << 30, [12], codeword=True)),
            ("codeword", lambda: decode_cfg(9, 3, 11, 9 * (256 << 20), [0])),
            ("codeword", lambda: decode_cfg(9, 3, 11, 9 * (256 << 20), [0], codeword=True)),
            ("repair", lambda: repair_cfg(9, 3, 11, 268_435_458, 0)),
            ("repair", lambda: repair_cfg(9, 3, 11, 268_435_458, 11)),
            ("repair", lambda: repair_cfg(10, 4, 13, 107_374_592, 0)),
            # alignment sensitivity: sub-chunk 3,314,048 (64-byte aligned rows) vs 3,314,018
            ("repair_align", lambda: repair_cfg(9, 3, 11, 81 * 3_314_048, 0))]
    for tag, fn in jobs:
        if tag in only:
            fn()

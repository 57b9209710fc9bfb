#!/usr/bin/env python3
"""Kernel time of (10,4,13) 1 GiB decodes of several erasure patterns on random chunks (HIP events
around each call on the launch stream, after a 150 ms prewarm): median / min ms per pattern and
the exec path.  CLAY_AMD_LIB picks the library build (same-box A/B of variants).
Usage: time_decode.py [pattern ...]   (pattern = comma-separated external node ids)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import clay_amd  # noqa: E402
from clay_amd import ClayCode  # noqa: E402

pats = [[int(x) for x in a.split(",")] for a in (sys.argv[1:] or ["0,4,8,12"])]
c = ClayCode(10, 4, 13)
chunk = c.encoded_chunk_size(1 << 30)
full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda")
outs = torch.empty((c.n, chunk), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
if os.environ.get("EXEC"):  # exec mode for the whole run (auto, stream-fused2, stream-local, grouped, ...)
    clay_amd.set_exec_mode(os.environ["EXEC"])
lib = os.path.basename(os.environ.get("CLAY_AMD_LIB", "libclay_amd.so"))
for er in pats:
    ins = [None if i in er else full[i] for i in range(c.n)]
    # DATA_ONLY=1: outputs for the erased data chunks only (what the reference's decode returns)
    ous = [outs[i] if i in er and (i < c.k or not os.environ.get("DATA_ONLY")) else None for i in range(c.n)]
    fn = lambda: c.decode_device(ins, er, ous, chunk, 0, st.cuda_stream)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) < 0.15:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    ms = []
    for _ in range(30):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    ms.sort()
    print(f"{lib} er={er} path={clay_amd.last_exec_path()} median {ms[15]:.4f} min {ms[0]:.4f} ms", flush=True)

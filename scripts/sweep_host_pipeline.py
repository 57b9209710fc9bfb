#!/usr/bin/env python3
"""Host-streaming encode (clay_encode_host_pipelined) on the BASELINE stripe: piece size x
stream count sweep, next to the raw pinned H2D / D2H copy rates that bound it.
Prints one JSON object per line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clay_amd import ClayCode  # noqa: E402

code = ClayCode(10, 4, 13)
chunk = code.encoded_chunk_size(1 << 30)
K, M = 10, 4
padded = K * chunk
hs = torch.randint(0, 256, (K, chunk), dtype=torch.uint8).pin_memory()
hp = torch.empty((M, chunk), dtype=torch.uint8).pin_memory()
dd = torch.empty((K, chunk), dtype=torch.uint8, device="cuda")
dp = torch.empty((M, chunk), dtype=torch.uint8, device="cuda")


def rate(fn, nbytes, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round(reps * nbytes / (time.perf_counter() - t0) / 2**30, 2)


print(json.dumps({"copy": "H2D pinned 10 chunks", "GiBps": rate(lambda: dd.copy_(hs, non_blocking=True), padded)}))
print(json.dumps({"copy": "D2H pinned 4 chunks", "GiBps": rate(lambda: hp.copy_(dp, non_blocking=True), M * chunk)}))
ref = None
for piece_mib in (8, 16, 32, 64, 128):
    for ns in (2, 3, 4):
        w = (piece_mib << 20) // (K * code.sub_chunk_no)
        r = rate(lambda: code.encode_host_pipelined([hs[i] for i in range(K)], [hp[j] for j in range(M)], chunk, 0,
                                                    w, ns), padded)
        if ref is None:
            ref = hp.clone()
        print(json.dumps({"piece_input_MiB": piece_mib, "streams": ns, "input_GiBps": r,
                          "same_parity": bool(torch.equal(hp, ref))}), flush=True)

#!/usr/bin/env python3
"""(4,2,5) encode of ~64 MiB stripes at power-of-two and skewed sub-chunk sizes: does the
2 MiB sub-chunk stride cost bandwidth?  Device-resident, HIP events."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clay_amd import ClayCode, last_encode_path  # noqa: E402

c = ClayCode(4, 2, 5)
st = torch.cuda.current_stream()
for sc in (2 << 20, (2 << 20) + 1024, (2 << 20) + 4096, (2 << 20) - 2048, 3 << 19, 1 << 21 | 1 << 19):
    chunk = sc * c.sub_chunk_no
    data = torch.randint(0, 256, (4, chunk), dtype=torch.uint8, device="cuda")
    par = torch.empty((2, chunk), dtype=torch.uint8, device="cuda")
    ts = []
    for i in range(25):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        c.encode_device([data[j] for j in range(4)], [par[j] for j in range(2)], chunk, 0, st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        if i >= 5:
            ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    print(f"sc {sc:>9} ({sc / 2**20:.4f} MiB) {ms:.4f} ms {6 * chunk / ms / 1e9:.0f} GB/s {last_encode_path()}", flush=True)

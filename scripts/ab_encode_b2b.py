#!/usr/bin/env python3
"""A/B encode variants on the BASELINE stripe the way bench.py times them: K back-to-back
launches on one stream, per-launch HIP events, mean; variants interleaved over rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import clay_amd  # noqa: E402
from clay_amd import ClayCode  # noqa: E402

variants = [(v.split(":")[0], int(v.split(":")[1]) if ":" in v else 0) for v in sys.argv[1:]] or [("stream", 0)]
code = ClayCode(10, 4, 13)
chunk = code.encoded_chunk_size(1 << 30)
data = torch.randint(0, 256, (10, chunk), dtype=torch.uint8, device="cuda")
par = torch.empty((4, chunk), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
res = {f"{v}:{t}": [] for v, t in variants}
ref = None
for rnd in range(4):
    for v, t in variants:
        clay_amd.set_encode_path(v, t)
        for _ in range(3):
            code.encode_device([data[i] for i in range(10)], [par[i] for i in range(4)], chunk, 0, st.cuda_stream)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        torch.cuda.synchronize()
        for a, b in evs:
            a.record(st)
            code.encode_device([data[i] for i in range(10)], [par[i] for i in range(4)], chunk, 0, st.cuda_stream)
            b.record(st)
        torch.cuda.synchronize()
        if ref is None:
            ref = par.clone()
        assert torch.equal(par, ref), (v, t)
        if rnd:
            res[f"{v}:{t}"] += [a.elapsed_time(b) for a, b in evs]
print(json.dumps({k: {"mean_ms": round(float(np.mean(x)), 4), "median_ms": round(float(np.median(x)), 4)}
                  for k, x in res.items()}))

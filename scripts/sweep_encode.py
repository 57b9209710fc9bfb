#!/usr/bin/env python3
"""A/B the encode paths on the BASELINE stripe in ONE process, interleaved rounds
(cdna_hip_programming.md rule 24).  Prints median/min kernel ms and GB/s per variant."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import clay_amd  # noqa: E402
from clay_amd import ClayCode  # noqa: E402

VARIANTS = [("bitsliced", 1), ("bitsliced", 2), ("bitsliced", 4), ("fused", 0)]
if len(sys.argv) > 1:
    VARIANTS = [(v.split(":")[0], int(v.split(":")[1]) if ":" in v else 0) for v in sys.argv[1:]]
code = ClayCode(10, 4, 13)
chunk = code.encoded_chunk_size(1 << 30)
data = torch.randint(0, 256, (10, chunk), dtype=torch.uint8, device="cuda")
outs = {v: torch.empty((4, chunk), dtype=torch.uint8, device="cuda") for v in VARIANTS}
stream = torch.cuda.current_stream()
algo = 14 * chunk
times = {v: [] for v in VARIANTS}
for rnd in range(12):
    for v in VARIANTS:
        clay_amd.set_encode_path(v[0], v[1])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        code.encode_device([data[i] for i in range(10)], [outs[v][i] for i in range(4)], chunk, 0,
                           stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if rnd >= 2:
            times[v].append(e0.elapsed_time(e1))
ref = outs[VARIANTS[0]].cpu()
res = {}
for v in VARIANTS:
    t = np.array(times[v])
    res[f"{v[0]}:{v[1]}"] = {"median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                            "GBps": round(algo / (np.median(t) * 1e-3) / 1e9, 1),
                            "same_as_first": bool(torch.equal(outs[v].cpu(), ref))}
print(json.dumps(res, indent=1))

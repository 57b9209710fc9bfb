#!/usr/bin/env python3
"""Minimal driver for rocprofv3: N encodes of the BASELINE 1 GiB (10,4,13) stripe on one path."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import clay_amd  # noqa: E402
from clay_amd import ClayCode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--path", default="auto")
ap.add_argument("--tile", type=int, default=0)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
code = ClayCode(10, 4, 13)
chunk = code.encoded_chunk_size(1 << 30)
data = torch.randint(0, 256, (10, chunk), dtype=torch.uint8, device="cuda")
par = torch.empty((4, chunk), dtype=torch.uint8, device="cuda")
clay_amd.set_encode_path(a.path, a.tile)
for _ in range(a.iters):
    code.encode_device([data[i] for i in range(10)], [par[i] for i in range(4)], chunk, 0,
                       torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print(clay_amd.last_encode_path())

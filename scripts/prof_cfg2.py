#!/usr/bin/env python3
"""(4,2,5) 64 MiB encode + single-erasure decode {0}, N back-to-back iterations each, for rocprofv3
kernel traces / PMC passes of the line-local kernels (bitslice_line.hpp)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from clay_amd import ClayCode  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()
c = ClayCode(4, 2, 5)
chunk = c.encoded_chunk_size(64 << 20)
full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda")
out = torch.empty(chunk, dtype=torch.uint8, device="cuda")
for _ in range(args.iters):
    c.encode_device([full[i] for i in range(c.k)], [full[c.k + x] for x in range(c.m)], chunk)
for _ in range(args.iters):
    c.decode_device([None if i == 0 else full[i] for i in range(c.n)], [0], [out if i == 0 else None for i in range(c.n)], chunk)
torch.cuda.synchronize()
print("done", flush=True)

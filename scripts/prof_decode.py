#!/usr/bin/env python3
"""One decode (10,4,13) 1 GiB with erasures --er (default {0,4,8,12}) (and optionally repair (9,3,11)),
repeated --iters times, for rocprofv3 --pmc passes (HBM bytes per launch; CLAY_EXEC picks the
executor: auto = the fused decode v2 for {0,4,8,12} (one erasure per section), else the grouped
executor / bs-repair; stream = streaming decode for every eligible pattern)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import clay_amd  # noqa: E402
from clay_amd import ClayCode  # noqa: E402

clay_amd.set_exec_mode(os.environ.get("CLAY_EXEC", "auto"))  # auto | grouped | tile | stream

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=4)
ap.add_argument("--what", default="decode4")
ap.add_argument("--er", default="0,4,8,12", help="erasures of the decode (e.g. 0 for the local decode)")
ap.add_argument("--prewarm-ms", type=float, default=0.0,
                help="back-to-back calls for this long first (the idle GPU's clock ramp; a trace "
                     "summary then skips them: scripts/trace_summary.py --skip)")
args = ap.parse_args()
if args.what == "decode4":
    c = ClayCode(10, 4, 13)
    chunk = c.encoded_chunk_size(1 << 30)
    er = [int(x) for x in args.er.split(",")]
    full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda")
    outs = torch.empty((c.n, chunk), dtype=torch.uint8, device="cuda")
    ins = [None if i in er else full[i] for i in range(c.n)]
    # DATA_ONLY=1: outputs for the erased data chunks only (what the reference's decode returns)
    ous = [outs[i] if i in er and (i < c.k or not os.environ.get("DATA_ONLY")) else None for i in range(c.n)]
    fn = lambda: c.decode_device(ins, er, ous, chunk)  # noqa: E731
else:
    c = ClayCode(9, 3, 11)
    chunk = 268_435_458
    sc = chunk // c.sub_chunk_no
    info = c.minimum_to_repair(0, list(range(1, 12)))
    hs = [h for h, _ in info]
    hb = torch.randint(0, 256, (len(hs), len(info[0][1]) * sc), dtype=torch.uint8, device="cuda")
    out = torch.empty(chunk, dtype=torch.uint8, device="cuda")
    fn = lambda: c.repair_device(0, hs, [hb[i] for i in range(len(hs))], chunk, out)  # noqa: E731
nwarm = 0
if args.prewarm_ms > 0:
    import time
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.prewarm_ms:
        for _ in range(8):
            fn()
        nwarm += 8
        torch.cuda.synchronize()
    nwarm += 1
for _ in range(args.iters):
    fn()
torch.cuda.synchronize()
print("done", args.what, args.iters, "prewarm_calls", nwarm)

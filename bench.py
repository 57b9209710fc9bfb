#!/usr/bin/env python3
"""Benchmark: device-resident Clay encode GiB/s at (k=10, m=4, d=13) -- BASELINE.json metric.

One step = encode of one 1 GiB stripe (the reference's ClayCode::encode of
1,073,741,824 bytes pads to 1,073,745,920 = 10 chunks of 107,374,592 bytes)
whose data chunks are already resident in HBM; parity (4 chunks) is written to
HBM.  Multi-GPU: one process per GPU (torchrun), each rank encodes its own
stripe (stripes are independent -> no data-path collective; weak scaling).  The
barrier / max-time reduction are timing plumbing only.

value       = stripes * padded stripe bytes / max-over-ranks wall time, GiB/s
roofline    = algorithmic bytes per launch (read 10 + write 4 chunks =
              1,503,244,288 B) / mean kernel time (HIP events on the launch
              stream) vs 8 TB/s HBM peak
cpu_baseline= the oracle (C restatement of the reference CPU path: scalar
              PRT/PFT + AVX2 RS region multiply, single thread) on a bounded
              sample of the same workload.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K, M, D = 10, 4, 13
STRIPE_BYTES = 1 << 30  # reference ClayCode::encode input
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prewarm-ms", type=float, default=250.0,
                    help="untimed encodes for this long before the warmup steps, so the timed "
                         "steps see the GPU at its sustained clock (an idle MI355X needs ~0.1 s of "
                         "load to ramp: 5 warmups gave 0.44 ms/launch, 200 gave 0.385)")
    ap.add_argument("--stripe-bytes", type=int, default=STRIPE_BYTES)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bound on the CPU-baseline sample (0 disables)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--path", default="auto",
                    choices=["auto", "fused", "staged", "bitsliced", "bitsliced2", "bitsliced3", "bitsliced4", "bitsliced5", "bitsliced6"])
    return ap.parse_args()


def latest_traffic():
    """Per-launch HBM bytes from the newest committed PMC summary (profiles/*_pmc.json)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*encode*_pmc.json")))
    if not files:
        return None, None
    try:
        with open(files[-1]) as f:
            j = json.load(f)
        return j.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)
    except Exception:
        return None, None


def cpu_baseline_threads(seconds: float, threads: int):
    """Stripe-parallel oracle encode on `threads` host cores (the reference
    itself is single-threaded; this is the all-cores CPU figure beside it)."""
    import threading
    from oracle import oracle  # checker/baseline only
    c = oracle.OracleClay(K, M, D)
    sample = 64 << 20
    data = np.random.default_rng(1).integers(0, 256, sample, dtype=np.uint8)
    c.encode_array(data)  # warm (lazy GF tables) before threads start
    counts = [0] * threads
    stop = time.perf_counter() + seconds

    def work(i):
        while time.perf_counter() < stop:
            c.encode_array(data)
            counts[i] += 1

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    padded = c.encoded_chunk_size(sample) * K
    n = sum(counts)
    return {"value": round(n * padded / el / 2**30, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n} x (10,4,13) encode of 64 MiB stripes on {threads} threads in {el:.1f}s, "
                      f"oracle/clay_oracle.c via ctypes (GIL released)"}


def cpu_baseline(seconds: float):
    from oracle import oracle  # checker/baseline only
    oracle.build()
    c = oracle.OracleClay(K, M, D)
    sample = 64 << 20  # 64 MiB stripes of the same code, repeated
    data = np.random.default_rng(1).integers(0, 256, sample, dtype=np.uint8)
    c.encode_array(data)  # warm
    n, t0 = 0, time.perf_counter()
    while True:
        c.encode_array(data)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    padded = c.encoded_chunk_size(sample) * K
    return {"value": round(n * padded / el / 2**30, 4), "unit": "GiB/s", "cores": 1,
            "kind": "port",
            "sample": f"{n} x (10,4,13) encode of 64 MiB stripes in {el:.1f}s, single thread, "
                      f"oracle/clay_oracle.c (scalar PRT/PFT + AVX2 RS, as reed-solomon-erasure simd-accel)"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import clay_amd
    from clay_amd import ClayCode
    clay_amd.set_encode_path(args.path)
    code = ClayCode(K, M, D)
    chunk = code.encoded_chunk_size(args.stripe_bytes)
    padded = chunk * K
    sc = chunk // code.sub_chunk_no

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    data = torch.randint(0, 256, (K, chunk), dtype=torch.uint8, device=dev, generator=g)
    par = torch.empty((M, chunk), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    dptr = [data[i] for i in range(K)]
    pptr = [par[i] for i in range(M)]

    t_pre = time.perf_counter()
    while (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
        for _ in range(8):
            code.encode_device(dptr, pptr, chunk, local, sh)
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        code.encode_device(dptr, pptr, chunk, local, sh)
    path = clay_amd.last_encode_path()
    launches = clay_amd.last_launch_count()
    torch.cuda.synchronize(dev)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        code.encode_device(dptr, pptr, chunk, local, sh)
        evs[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tmax = float(t.item())

    verified = None
    if rank == 0 and world == 1 and not args.no_verify:
        from oracle import oracle
        oracle.build()
        host = data.cpu().numpy().reshape(-1)
        ref = oracle.OracleClay(K, M, D).encode_array(host[:padded])
        verified = bool(np.array_equal(par.cpu().numpy(), ref[K:]))

    host_incl = host_sync = None
    if rank == 0 and world == 1 and not args.no_host_path:
        # PCIe-inclusive: pinned host data chunks -> device -> parity back to pinned
        # host memory.  host_sync: one stream, whole-stripe copies; host_incl: the pipelined
        # host-streaming encode (clay_encode_host_pipelined, pieces over 3 streams).
        hsrc = torch.empty((K, chunk), dtype=torch.uint8).pin_memory()
        hdst = torch.empty((M, chunk), dtype=torch.uint8).pin_memory()
        hsrc.copy_(data.cpu())
        reps = 3
        torch.cuda.synchronize(dev)
        h0 = time.perf_counter()
        for _ in range(reps):
            data.copy_(hsrc, non_blocking=True)
            code.encode_device(dptr, pptr, chunk, local, sh)
            hdst.copy_(par, non_blocking=True)
        torch.cuda.synchronize(dev)
        host_sync = round(reps * padded / (time.perf_counter() - h0) / 2**30, 3)
        hs, hd = [hsrc[i] for i in range(K)], [hdst[i] for i in range(M)]
        code.encode_host_pipelined(hs, hd, chunk, local)  # warm (streams, piece buffers)
        h0 = time.perf_counter()
        for _ in range(reps):
            code.encode_host_pipelined(hs, hd, chunk, local)
        host_incl = round(reps * padded / (time.perf_counter() - h0) / 2**30, 3)
        if verified is not None:
            verified = verified and bool(torch.equal(hdst, par.cpu()))

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    algo_bytes = padded + M * chunk  # read k chunks + write m chunks per launch
    mean_ms = float(np.mean(kern_ms))
    achieved = algo_bytes / (mean_ms * 1e-3) / 1e9
    traffic, traffic_src = latest_traffic()
    out = {
        "metric": "device-resident encode GiB/s at (k=10,m=4,d=13); % of HBM roofline",
        "value": round(world * args.steps * padded / tmax / 2**30, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(tmax / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (uniform random bytes, torch generator seed 1234+rank), device-resident",
        "config": {"workload": "(k=10,m=4,d=13) encode, one 1 GiB stripe per GPU",
                   "stripe_input_bytes": args.stripe_bytes, "padded_stripe_bytes": padded,
                   "chunk_bytes": chunk, "sub_chunk_bytes": sc, "alpha": code.sub_chunk_no,
                   "parallelism": f"stripe-per-gpu x{world}", "encode_path": path,
                   "launches_per_step": launches, "prewarm_ms": args.prewarm_ms},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_ms_mean": round(mean_ms, 4), "kernel_ms_min": round(min(kern_ms), 4)},
        "verified_vs_oracle": verified,
        "host_inclusive_GiBps": host_incl,
        "host_inclusive_sync_GiBps": host_sync,
    }
    if world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        out["cpu_baseline_all_cores"] = cpu_baseline_threads(args.cpu_seconds / 2,
                                                             min(16, os.cpu_count() or 1))
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Benchmark: device-resident Clay encode GiB/s at (k=10, m=4, d=13) -- BASELINE.json metric.

One step = encode of one 1 GiB stripe (the reference's ClayCode::encode of
1,073,741,824 bytes pads to 1,073,745,920 = 10 chunks of 107,374,592 bytes)
whose data chunks are already resident in HBM; parity (4 chunks) is written to
HBM.  Multi-GPU: one process per GPU, each rank encodes its own stripe (stripes
are independent, encode.rs:30-80 -> no data-path collective; weak scaling).  The
barrier / max-time reduction are timing plumbing only and run over gloo (no RCCL).

    python bench.py                      # N = 1
    python bench.py --gpus 8             # spawns 8 ranks itself (no torchrun needed)
    torchrun --nproc-per-node 8 bench.py --gpus 8   # same, launched externally

value       = ranks * padded stripe bytes * steps / max-over-ranks wall time, GiB/s
roofline    = algorithmic bytes per launch (read 10 + write 4 chunks =
              1,503,244,288 B) / mean kernel time (HIP events on the launch
              stream) vs 8 TB/s HBM peak
cpu_baseline= the oracle (C restatement of the reference CPU path: scalar
              PRT/PFT + AVX2 RS region multiply, single thread) on a bounded
              sample of the same workload, rank 0 at N = 1 only; cfg1 adds the
              reference's own bench shape, (4,2,5) on 1 MiB (clay_bench.rs:20-56).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K, M, D = 10, 4, 13
STRIPE_BYTES = 1 << 30  # reference ClayCode::encode input
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
# best copy kernel measured on this pool: LDS-DMA loader waves + writer waves per CU, nt stores
# (bench_tools/bw_probe.hip, profiles/r03/bw_probe_r03.txt; the encode's own 5:2 read/write mix
# streams at 5,090 GB/s with plain loads/stores in the same sweep)
COPY_CEILING_GBS = 5546.0
VERIFY_W = 4096         # positions per verified column slice (every rank, both ends)


def parse(argv=None):
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
                    help="bound on the headline CPU-baseline sample (0 disables all CPU legs)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-small", action="store_true", help="skip the clay_bench-size GPU batch rates")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the driver-timed legs of BASELINE configs 2, 3 and 5 (after the timed region)")
    ap.add_argument("--leg-calls", type=int, default=30, help="timed calls per config leg")
    ap.add_argument("--path", default="auto",
                    choices=["auto", "fused", "staged", "bitsliced", "stream"])
    ap.add_argument("--tile", type=int, default=0, help="encode path variant (clay_set_encode_path)")
    ap.add_argument("--launch-timeout", type=float, default=900.0,
                    help="--gpus N launcher: stop every rank after this many seconds (0 = no limit)")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="torch.distributed timeout (s) for init and collectives")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # launcher tests
    ap.add_argument("--cpu-dry", action="store_true",
                    help="test mode without a GPU: the oracle replaces the device encode; everything "
                         "else (launcher, ranks, gloo timing plane, JSON) is the same")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: `--gpus N` without an external torchrun spawns N fresh rank processes
# before this process touches HIP (never exec from a GPU-initialised process)
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv) -> int:
    """Spawn one rank process per GPU and supervise them: every rank is polled, and the
    first rank that exits non-zero (bad ordinal, OOM, a fault) takes the others down at
    once instead of leaving them blocked in a barrier -- the launcher then exits with that
    rank's code.  The parent never touches HIP."""
    port = _free_port()
    # build the CPU checker once here (CPU only, no HIP) so the ranks never race on make
    from oracle import oracle
    oracle.build()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(args.gpus),
                    "LOCAL_WORLD_SIZE": str(args.gpus), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    deadline = time.monotonic() + args.launch_timeout if args.launch_timeout > 0 else None
    rc = 0
    live = set(range(len(procs)))
    while live:
        for r in sorted(live):
            code = procs[r].poll()
            if code is None:
                continue
            live.discard(r)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
        if rc != 0 or (deadline is not None and time.monotonic() > deadline):
            if rc == 0:
                rc = 124
                print(f"bench: ranks still running after {args.launch_timeout:.0f} s; stopping them",
                      file=sys.stderr, flush=True)
            for r in live:
                procs[r].terminate()
            for r in live:
                try:
                    procs[r].wait(timeout=10)
                except subprocess.TimeoutExpired:
                    procs[r].kill()
                    procs[r].wait()
            break
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------
# CPU baselines (oracle = the reference CPU path restated in C; checker / baseline only)
# ---------------------------------------------------------------------------
def host_info() -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=5).stdout.strip())
    except Exception:
        nproc = None
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "nproc": nproc,
            "affinity_cpus": affinity, "omp_num_threads": int(omp) if omp and omp.isdigit() else None}


def all_cores_threads(info: dict) -> int:
    """Threads for the all-cores CPU figure: the CPUs this process may run on, bounded by the
    box's CPU share (OMP_NUM_THREADS is set to it on the GPU pool)."""
    n = info["affinity_cpus"] or 1
    if info["omp_num_threads"]:
        n = min(n, info["omp_num_threads"])
    return max(1, n)


def _timed(fn, seconds: float, threads: int = 1):
    """Run fn() repeatedly on `threads` threads for ~`seconds`; returns (calls, elapsed)."""
    import threading
    counts = [0] * threads
    stop = time.perf_counter() + seconds

    def work(i):
        while time.perf_counter() < stop:
            fn()
            counts[i] += 1

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return sum(counts), time.perf_counter() - t0


def cpu_baseline_headline(seconds: float, threads: int):
    """(10,4,13) encode on 64 MiB stripes of the same code: the reference is single-threaded
    (no threads in the crate); the all-cores figure runs independent stripes in parallel
    (ctypes releases the GIL)."""
    from oracle import oracle  # checker / baseline only
    oracle.build()
    c = oracle.OracleClay(K, M, D)
    sample = 64 << 20
    data = np.random.default_rng(1).integers(0, 256, sample, dtype=np.uint8)
    c.encode_array(data)  # warm (lazy GF tables)
    padded = c.encoded_chunk_size(sample) * K
    n1, e1 = _timed(lambda: c.encode_array(data), seconds, 1)
    nt, et = _timed(lambda: c.encode_array(data), seconds / 2, threads)
    one = {"value": round(n1 * padded / e1 / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
           "sample": f"{n1} x (10,4,13) encode of 64 MiB stripes in {e1:.1f}s, single thread, "
                     f"oracle/clay_oracle.c (scalar PRT/PFT + AVX2 RS, as reed-solomon-erasure simd-accel)"}
    allc = {"value": round(nt * padded / et / 2**30, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{nt} x (10,4,13) encode of 64 MiB stripes on {threads} threads in {et:.1f}s"}
    return one, allc


def cpu_baseline_cfg1(seconds: float, threads: int):
    """BASELINE.json configs[0]: ClayCode::encode of 1 MiB at (4,2,5) on the reference CPU path
    (the criterion shape of benches/clay_bench.rs:20-56, data from a fixed seed), plus the same
    file's decode (1 erasure, node 0, :58-93) and repair (node 0, :95-138) legs.  Throughput is
    input bytes per second, as criterion's Throughput::Bytes(size)."""
    from oracle import oracle
    oracle.build()
    k, m, d = 4, 2, 5
    size = 1 << 20
    c = oracle.OracleClay(k, m, d)
    data = np.random.default_rng(42).integers(0, 256, size, dtype=np.uint8)
    enc = c.encode_array(data)
    chunk = enc.shape[1]
    avail = {i: enc[i] for i in range(1, c.n)}
    info = c.minimum_to_repair(0, list(range(1, c.n)))
    sc = chunk // c.sub_chunk_no
    helper = {h: np.concatenate([enc[h][z * sc:(z + 1) * sc] for z in idx]) for h, idx in info}
    legs = {"encode": lambda: c.encode_array(data),
            "decode_1_erasure": lambda: c.decode(avail, [0]),
            "repair_node0": lambda: c.repair(0, helper, chunk)}
    out = {"config": "(k=4,m=2,d=5) 1 MiB (clay_bench.rs shape), oracle/clay_oracle.c", "unit": "MiB/s",
           "chunk_bytes": chunk, "sub_chunk_bytes": sc}
    per = max(0.5, seconds / (2 * len(legs)))
    for name, fn in legs.items():
        fn()
        n1, e1 = _timed(fn, per, 1)
        nt, et = _timed(fn, per, threads)
        out[name] = {"single_thread": round(n1 * size / e1 / 2**20, 2),
                     "all_cores": round(nt * size / et / 2**20, 2), "cores": threads,
                     "calls": [n1, nt], "seconds": [round(e1, 2), round(et, 2)]}
    return out


# ---------------------------------------------------------------------------
# GPU legs
# ---------------------------------------------------------------------------
def verify_slices(code, data, par, chunk, oracle_cls):
    """Parity of positions [0, w) and [sc - w, sc) of every sub-chunk against the oracle: each
    byte offset is an independent codeword, so a column slice is a small stripe of its own."""
    alpha = code.sub_chunk_no
    sc = chunk // alpha
    w = min(VERIFY_W, sc)
    o = oracle_cls(K, M, D)
    ok = True
    for p0 in sorted({0, sc - w}):
        d = data.view(K, alpha, sc)[:, :, p0:p0 + w].contiguous().cpu().numpy().reshape(-1)
        ref = o.encode_array(d)
        got = par.view(M, alpha, sc)[:, :, p0:p0 + w].contiguous().cpu().numpy().reshape(M, -1)
        ok = ok and bool(np.array_equal(got, ref[K:]))
    return ok


def small_stripe_rates(torch, dev, local, sh):
    """GPU batched encode at the reference bench sizes (clay_bench.rs:20-25, (4,2,5)): many
    independent stripes per call through clay_encode_device_batch, device-resident."""
    from clay_amd import ClayCode
    import clay_amd
    code = ClayCode(4, 2, 5)
    out = {"config": "(k=4,m=2,d=5) clay_encode_device_strided ([n][k][chunk] buffers), ~64 MiB of input per call",
           "unit": "GiB/s"}
    for size in (1024, 10 * 1024, 100 * 1024, 1 << 20):
        chunk = code.encoded_chunk_size(size)
        n = max(4, (64 << 20) // (4 * chunk))
        data = torch.randint(0, 256, (n * 4, chunk), dtype=torch.uint8, device=dev)
        par = torch.empty((n * 2, chunk), dtype=torch.uint8, device=dev)
        for _ in range(3):
            code.encode_device_strided(data, par, n, chunk, device=local, stream=sh)
        torch.cuda.synchronize(dev)
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            code.encode_device_strided(data, par, n, chunk, device=local, stream=sh)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        out[f"{size}B"] = {"stripes_per_call": n, "GiBps": round(reps * n * size / el / 2**30, 2),
                           "us_per_call": round(el / reps * 1e6, 1), "path": clay_amd.last_encode_path()}
        del data, par
    return out


def _event_times(torch, stream, fn, calls: int, warm: int = 10, prewarm_ms: float = 150.0):
    """HIP-event time of each of `calls` back-to-back calls on `stream` (events recorded on the
    launch stream, all calls queued before one synchronize), after `warm` untimed calls and
    untimed calls for `prewarm_ms` (the GPU idles while the previous leg's oracle check runs, and
    an idle MI355X needs ~0.1 s of load to return to its sustained clock -- without this the
    first leg after a check read 0.39 ms for a 0.35 ms kernel)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < prewarm_ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def _leg(name, ms, algo, path, verified, extra=None):
    mean = float(np.mean(ms))
    d = {"workload": name, "kernel_ms_mean": round(mean, 4), "kernel_ms_median": round(float(np.median(ms)), 4),
         "kernel_ms_min": round(float(min(ms)), 4),
         "calls": len(ms), "algorithmic_bytes": int(algo), "achieved_GBps": round(algo / (mean * 1e-3) / 1e9, 1),
         "frac": round(algo / (mean * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "path": path, "verified_vs_oracle": verified}
    if extra:
        d.update(extra)
    return d


def _slice_cols(arr2d, alpha, p0, w):
    """Columns [p0, p0 + w) of every sub-chunk of each row of a (rows, alpha * sc) device tensor,
    as a host array (rows, alpha * w): an independent smaller instance of the same code."""
    rows = arr2d.shape[0]
    sc = arr2d.shape[1] // alpha
    return arr2d.view(rows, alpha, sc)[:, :, p0:p0 + w].contiguous().cpu().numpy().reshape(rows, alpha * w)


def config_legs(torch, dev, local, stream, oracle_cls, calls: int):
    """Driver-timed legs for the other BASELINE GPU configs (and
    the single-erasure decode of config 5's stripe),
    each run AFTER the encode's timed region on fresh device buffers: HIP-event kernel time per
    call, the §8(d) algorithmic bytes, the fraction of 8 TB/s, the kernel path, and a column-slice
    check against the oracle (every byte offset of the sub-chunks is an independent codeword, so
    positions [p0, p0 + w) of every sub-chunk form a small instance of the same call)."""
    import clay_amd
    from clay_amd import ClayCode
    sh = stream.cuda_stream
    out = {}
    g = torch.Generator(device=dev)

    def rnd(shape, seed):
        g.manual_seed(seed)
        return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=g)

    # config 5: (10,4,13) 1 GiB stripe, 4 erasures {0,4,8,12} (worst case), random chunks
    c = ClayCode(10, 4, 13)
    chunk = c.encoded_chunk_size(1 << 30)
    alpha, sc = c.sub_chunk_no, chunk // c.sub_chunk_no
    er = [0, 4, 8, 12]
    full = rnd((c.n, chunk), 51)
    outs = torch.zeros((c.n, chunk), dtype=torch.uint8, device=dev)
    ins = [None if i in er else full[i] for i in range(c.n)]
    # the reference's decode returns the data chunks (decode.rs:167-257): the erased parity chunk
    # is solved for inside the kernel but not written
    ous = [outs[i] if i in er and i < c.k else None for i in range(c.n)]
    ms = _event_times(torch, stream, lambda: c.decode_device(ins, er, ous, chunk, local, sh), calls)
    path = clay_amd.last_exec_path()
    o = oracle_cls(10, 4, 13)
    ok = True
    for p0 in (0, sc - VERIFY_W):
        s = _slice_cols(full, alpha, p0, VERIFY_W)
        got = _slice_cols(outs, alpha, p0, VERIFY_W)
        ref = np.frombuffer(o.decode({i: s[i] for i in range(c.n) if i not in er}, er), np.uint8).reshape(10, -1)
        ok = ok and all(np.array_equal(got[e], ref[e]) for e in er if e < 10)
    algo = (c.n - len(er)) * chunk + sum(1 for e in er if e < 10) * chunk
    out["decode_cfg5"] = _leg("(k=10,m=4,d=13) decode, 1 GiB stripe, erasures {0,4,8,12}, random chunks",
                              ms, algo, path, ok, {"bytes_counted": "10 survivors read + 3 erased data chunks written"})
    # the same stripe with one erasure {0} (the common case: the local decode on 256-byte runs)
    er = [0]
    ins = [None if i in er else full[i] for i in range(c.n)]
    ous = [outs[i] if i in er else None for i in range(c.n)]
    ms = _event_times(torch, stream, lambda: c.decode_device(ins, er, ous, chunk, local, sh), calls)
    path = clay_amd.last_exec_path()
    ok = True
    for p0 in (0, sc - VERIFY_W):
        s = _slice_cols(full, alpha, p0, VERIFY_W)
        got = _slice_cols(outs, alpha, p0, VERIFY_W)
        ref = np.frombuffer(o.decode({i: s[i] for i in range(c.n) if i not in er}, er), np.uint8).reshape(10, -1)
        ok = ok and np.array_equal(got[0], ref[0])
    algo = (c.n - 1) * chunk + chunk
    out["decode_1erasure"] = _leg("(k=10,m=4,d=13) decode, 1 GiB stripe, erasure {0}, random chunks",
                                  ms, algo, path, ok, {"bytes_counted": "13 survivors read + 1 erased data chunk written"})
    del full, outs, ins, ous

    # config 3: (9,3,11) repair of node 0 from d = 11 helpers, chunk 268,435,458 (beta sub-chunks each)
    c = ClayCode(9, 3, 11)
    chunk = 268_435_458
    alpha, sc = c.sub_chunk_no, chunk // c.sub_chunk_no
    info = c.minimum_to_repair(0, [i for i in range(c.n) if i != 0])
    helpers, idx = [h for h, _ in info], info[0][1]
    beta = len(idx)
    hb = rnd((len(helpers), beta * sc), 31)
    rep = torch.zeros(chunk, dtype=torch.uint8, device=dev)
    hl = [hb[i] for i in range(len(helpers))]
    ms = _event_times(torch, stream, lambda: c.repair_device(0, helpers, hl, chunk, rep, local, sh), calls)
    path = clay_amd.last_exec_path()
    o = oracle_cls(9, 3, 11)
    ok = True
    for p0 in (0, sc - VERIFY_W):
        hs = _slice_cols(hb, beta, p0, VERIFY_W)
        got = _slice_cols(rep.view(1, -1), alpha, p0, VERIFY_W)[0]
        ref = o.repair(0, {h: hs[j] for j, h in enumerate(helpers)}, alpha * VERIFY_W)
        ok = ok and np.array_equal(got, np.frombuffer(ref, np.uint8))
    algo = len(helpers) * beta * sc + chunk
    out["repair_cfg3"] = _leg("(k=9,m=3,d=11) repair of node 0 from 11 helpers, chunk 268,435,458",
                              ms, algo, path, ok, {"bytes_counted": "d x beta x sc read + the chunk written"})
    del hb, rep, hl

    # config 2: (4,2,5) 64 MiB stripe: encode, then decode of erasure {0}
    c = ClayCode(4, 2, 5)
    chunk = c.encoded_chunk_size(64 << 20)
    alpha, sc = c.sub_chunk_no, chunk // c.sub_chunk_no
    full = torch.zeros((c.n, chunk), dtype=torch.uint8, device=dev)
    full[:4] = rnd((4, chunk), 21)
    dl, pl = [full[i] for i in range(4)], [full[4 + i] for i in range(2)]
    ms_e = _event_times(torch, stream, lambda: c.encode_device(dl, pl, chunk, local, sh), calls)
    epath = clay_amd.last_encode_path()
    o = oracle_cls(4, 2, 5)
    ok_e = True
    for p0 in (0, sc - VERIFY_W):
        s = _slice_cols(full, alpha, p0, VERIFY_W)
        ok_e = ok_e and np.array_equal(s[4:], o.encode_array(s[:4].reshape(-1))[4:])
    outs = torch.zeros((c.n, chunk), dtype=torch.uint8, device=dev)
    er = [0]
    ins = [None if i in er else full[i] for i in range(c.n)]
    ous = [outs[i] if i in er else None for i in range(c.n)]
    ms_d = _event_times(torch, stream, lambda: c.decode_device(ins, er, ous, chunk, local, sh), calls)
    dpath = clay_amd.last_exec_path()
    # oracle check on column slices, as the other legs (the survivors' slices through the
    # oracle's decode; ADVICE r05: not a self-consistency check against our own encode)
    ok_d = True
    for p0 in (0, sc - VERIFY_W):
        s = _slice_cols(full, alpha, p0, VERIFY_W)
        got = _slice_cols(outs, alpha, p0, VERIFY_W)
        ref = np.frombuffer(o.decode({i: s[i] for i in range(c.n) if i not in er}, er), np.uint8).reshape(4, -1)
        ok_d = ok_d and np.array_equal(got[0], ref[0])
    out["cfg2_encode"] = _leg("(k=4,m=2,d=5) encode, 64 MiB stripe", ms_e, 6 * chunk, epath, ok_e,
                              {"bytes_counted": "4 data chunks read + 2 parity written"})
    out["cfg2_decode"] = _leg("(k=4,m=2,d=5) decode of erasure {0}, 64 MiB stripe (a codeword)", ms_d,
                              5 * chunk + chunk, dpath, ok_d,
                              {"bytes_counted": "5 survivors read + 1 erased data chunk written"})
    del full, outs, ins, ous
    torch.cuda.synchronize()
    return out


def latest_traffic():
    """Per-launch HBM bytes from the newest committed PMC summary (profiles/*encode*_pmc.json)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*encode*_pmc.json")))
    if not files:
        return None, None
    try:
        with open(files[-1]) as f:
            j = json.load(f)
        return j.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)
    except Exception:
        return None, None


def run_rank(args) -> int:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import datetime

    import torch
    import torch.distributed as dist
    if rank == args.fail_rank:  # launcher test: this rank dies before the rendezvous
        print(f"bench: rank {rank} failing on request (--fail-rank)", file=sys.stderr, flush=True)
        return 3
    if not args.cpu_dry:
        ndev = torch.cuda.device_count()
        if local >= ndev:
            print(f"bench: LOCAL_RANK {local} but only {ndev} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    if world > 1:
        # gloo in every mode: the data path has no collective (whole stripes per GPU), and the
        # control plane -- the start / stop barrier and the all_gather of three doubles per rank
        # -- needs no RCCL bring-up across the node (north_star: "RCCL unused")
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.dist_timeout))
    from oracle import oracle  # checker / CPU legs only (and the dry run's stand-in encode)
    oracle.build()

    ocode = oracle.OracleClay(K, M, D)
    chunk = ocode.encoded_chunk_size(args.stripe_bytes)
    padded = chunk * K
    alpha = ocode.sub_chunk_no
    sc = chunk // alpha
    path, launches = "oracle-cpu-dry", 0
    verified = None

    if args.cpu_dry:
        host = np.random.default_rng(1234 + rank).integers(0, 256, padded, dtype=np.uint8)
        step = lambda: ocode.encode_array(host)  # noqa: E731
        sync = lambda: None  # noqa: E731
        dev_t = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        dev_t = torch.device("cuda", local)
        import clay_amd
        from clay_amd import ClayCode
        clay_amd.set_encode_path(args.path, args.tile)
        code = ClayCode(K, M, D)
        assert code.encoded_chunk_size(args.stripe_bytes) == chunk
        g = torch.Generator(device=dev_t)
        g.manual_seed(1234 + rank)
        data = torch.randint(0, 256, (K, chunk), dtype=torch.uint8, device=dev_t, generator=g)
        par = torch.empty((M, chunk), dtype=torch.uint8, device=dev_t)
        stream = torch.cuda.current_stream(dev_t)
        sh = stream.cuda_stream
        dptr = [data[i] for i in range(K)]
        pptr = [par[i] for i in range(M)]
        step = lambda: code.encode_device(dptr, pptr, chunk, local, sh)  # noqa: E731
        sync = lambda: torch.cuda.synchronize(dev_t)  # noqa: E731
        t_pre = time.perf_counter()
        while (time.perf_counter() - t_pre) * 1e3 < args.prewarm_ms:
            for _ in range(8):
                step()
            sync()

    for _ in range(args.warmup):
        step()
    sync()
    if not args.cpu_dry:
        path = clay_amd.last_encode_path()
        launches = clay_amd.last_launch_count()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]

    # ---- timed region: exactly K steps between barrier + synchronize on both sides ----
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if not args.cpu_dry:
            evs[i][0].record(stream)
        step()
        if not args.cpu_dry:
            evs[i][1].record(stream)
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if args.cpu_dry:
        kern_ms = [el / args.steps * 1e3] * args.steps
        verified = True
    else:
        kern_ms = [a.elapsed_time(b) for a, b in evs]
        if not args.no_verify:
            verified = verify_slices(code, data, par, chunk, oracle.OracleClay)

    # per-rank wall / kernel mean / verified -> every rank (max over ranks is the job time)
    mine = torch.tensor([el, float(np.mean(kern_ms)), 0.0 if verified is False else 1.0],
                        dtype=torch.float64)  # CPU tensor: the gloo group carries it
    if world > 1:
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per = [t.cpu().tolist() for t in allr]
    else:
        per = [mine.cpu().tolist()]
    tmax = max(p[0] for p in per)

    host_incl = host_sync = small = legs = None
    if rank == 0 and world == 1 and not args.cpu_dry:
        if not args.no_host_path:
            # PCIe-inclusive: pinned host data chunks -> device -> parity back to
            # pinned host memory.  host_sync: one stream, whole-stripe copies; host_incl: the
            # pipelined host-streaming encode (clay_encode_host_pipelined, pieces over 3 streams).
            hsrc = torch.empty((K, chunk), dtype=torch.uint8).pin_memory()
            hdst = torch.empty((M, chunk), dtype=torch.uint8).pin_memory()
            hsrc.copy_(data.cpu())
            reps = 3
            sync()
            h0 = time.perf_counter()
            for _ in range(reps):
                data.copy_(hsrc, non_blocking=True)
                step()
                hdst.copy_(par, non_blocking=True)
            sync()
            host_sync = round(reps * padded / (time.perf_counter() - h0) / 2**30, 3)
            hs, hd = [hsrc[i] for i in range(K)], [hdst[i] for i in range(M)]
            code.encode_host_pipelined(hs, hd, chunk, local)  # warm (streams, piece buffers)
            h0 = time.perf_counter()
            for _ in range(reps):
                code.encode_host_pipelined(hs, hd, chunk, local)
            host_incl = round(reps * padded / (time.perf_counter() - h0) / 2**30, 3)
            if verified is not None:
                verified = verified and bool(torch.equal(hdst, par.cpu()))
        if not args.no_small:
            small = small_stripe_rates(torch, dev_t, local, sh)
        if not args.no_legs:
            del data, par, dptr, pptr
            legs = config_legs(torch, dev_t, local, stream, oracle.OracleClay, args.leg_calls)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return 0

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
        "data": ("synthetic (uniform random bytes, seed 1234+rank), "
                 + ("host memory, oracle stand-in encode (--cpu-dry)" if args.cpu_dry else "device-resident")),
        "config": {"workload": "(k=10,m=4,d=13) encode, one 1 GiB stripe per GPU",
                   "stripe_input_bytes": args.stripe_bytes, "padded_stripe_bytes": padded,
                   "chunk_bytes": chunk, "sub_chunk_bytes": sc, "alpha": alpha,
                   "parallelism": f"stripe-per-gpu x{world}", "encode_path": path,
                   "launches_per_step": launches, "prewarm_ms": args.prewarm_ms},
        "per_rank": {"wall_ms_per_step": [round(p[0] / args.steps * 1e3, 4) for p in per],
                     "kernel_ms_mean": [round(p[1], 4) for p in per],
                     "verified": [bool(p[2]) for p in per]},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "measured_copy_ceiling": COPY_CEILING_GBS,
                     "frac_of_measured_copy": round(achieved / COPY_CEILING_GBS, 4),
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_ms_mean": round(mean_ms, 4), "kernel_ms_min": round(min(kern_ms), 4)},
        "verified_vs_oracle": verified if world == 1 else all(bool(p[2]) for p in per),
        "host_inclusive_GiBps": host_incl,
        "host_inclusive_sync_GiBps": host_sync,
        "gpu_small_stripes": small,
        "config_legs": legs,
    }
    if args.cpu_dry:
        out["cpu_dry"] = True
    if world == 1 and args.cpu_seconds > 0:
        info = host_info()
        threads = all_cores_threads(info)
        one, allc = cpu_baseline_headline(args.cpu_seconds, threads)
        out["cpu_baseline"] = one
        out["cpu_baseline_all_cores"] = allc
        out["cpu_baseline_cfg1"] = cpu_baseline_cfg1(min(args.cpu_seconds, 8.0), threads)
        out["host"] = info
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args, argv)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())

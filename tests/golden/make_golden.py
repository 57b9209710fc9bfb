#!/usr/bin/env python3
"""Generate the committed golden vectors (tests/golden/*.npz) with the oracle.

The reference holds no golden byte vectors and cannot be built here (no
cargo/rustc; reed-solomon-erasure 6.0.0 not vendored), so these fixtures are
produced by oracle/clay_oracle.c -- pinned by the KATs in tests/test_oracle_kats.py
and the reference property tests in tests/test_reference_properties.py.  They
freeze the oracle's bytes (regression pin) and give the GPU tests fixed vectors.
Inputs: seeded uniform bytes plus the reference tests' own data patterns
(i % 256, lib.rs:438; (i*7+13) % 256, lib.rs:467; (i*17+31) % 256, integration.rs:23).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle  # noqa: E402

CASES = [  # (k, m, d, data_len, pattern)
    (4, 2, 5, 1000, "rand"),
    (4, 2, 5, 4 * 8 * 2, "i%256"),
    (6, 3, 8, 6 * 27 * 2 * 3 + 5, "rand"),
    (9, 3, 11, 9 * 81, "(i*7+13)%256"),
    (9, 3, 11, 9 * 81 * 2 * 2, "rand"),
    (10, 4, 13, 10 * 256, "(i*17+31)%256"),
    (10, 4, 13, 10 * 256 * 2 * 6 + 77, "rand"),
    (5, 3, 6, 5 * 16 * 2 * 3, "rand"),
]


def data_for(n, pattern, seed):
    i = np.arange(n, dtype=np.int64)
    if pattern == "rand":
        return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
    return (eval(pattern.replace("%", " % "), {"i": i}) % 256).astype(np.uint8)


def main():
    for ci, (k, m, d, n, pat) in enumerate(CASES):
        c = oracle.OracleClay(k, m, d)
        data = data_for(n, pat, ci)
        enc = c.encode_array(data)
        chunk = enc.shape[1]
        sc = chunk // c.sub_chunk_no
        rng = np.random.default_rng(1000 + ci)
        out = {"k": k, "m": m, "d": d, "pattern": pat, "data": data, "encoded": enc}
        # decode of NON-codeword inputs for several erasure patterns (pins RS row choice)
        er_list = [[0], [c.n - 1], list(range(m)), [i * c.q for i in range(m) if i * c.q < c.n][:m]]
        for j, er in enumerate(er_list):
            noisy = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
            av = {i: noisy[i] for i in range(c.n) if i not in er}
            out[f"dec{j}_erasures"] = np.array(er)
            out[f"dec{j}_input"] = noisy
            out[f"dec{j}_output"] = np.frombuffer(c.decode(av, er), np.uint8)
        # repair of every node from random helper payloads
        for lost in range(c.n):
            info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
            hs = np.array([h for h, _ in info])
            payload = rng.integers(0, 256, (len(hs), len(info[0][1]) * sc), dtype=np.uint8)
            out[f"rep{lost}_helpers"] = hs
            out[f"rep{lost}_payload"] = payload
            out[f"rep{lost}_output"] = np.frombuffer(
                c.repair(lost, {int(h): payload[i] for i, h in enumerate(hs)}, chunk), np.uint8)
        path = os.path.join(HERE, f"clay_{k}_{m}_{d}_{ci}.npz")
        np.savez_compressed(path, **out)
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()

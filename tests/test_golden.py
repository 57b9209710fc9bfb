"""Committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py).
CPU: the oracle still reproduces them.  GPU: the HIP path reproduces them exactly."""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FILES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def load(path):
    return dict(np.load(path, allow_pickle=False))


def cases(g):
    c = int(g["k"]), int(g["m"]), int(g["d"])
    n = c[0] + c[1]
    decs = sorted({key.split("_")[0] for key in g if key.startswith("dec")})
    reps = [r for r in range(n) if f"rep{r}_output" in g]
    return c, n, decs, reps


def check(code, g):
    (k, m, d), n, decs, reps = cases(g)
    enc = g["encoded"]
    chunk = enc.shape[1]
    assert np.array_equal(np.asarray(code.encode_array(g["data"])), enc)
    for dk in decs:
        er = [int(x) for x in g[f"{dk}_erasures"]]
        noisy = g[f"{dk}_input"]
        av = {i: noisy[i] for i in range(n) if i not in er}
        assert np.frombuffer(code.decode(av, er), np.uint8).tobytes() == g[f"{dk}_output"].tobytes(), dk
    for r in reps:
        hs = [int(h) for h in g[f"rep{r}_helpers"]]
        pl = g[f"rep{r}_payload"]
        got = code.repair(r, {h: pl[i] for i, h in enumerate(hs)}, chunk)
        assert got == g[f"rep{r}_output"].tobytes(), r


def test_golden_files_present():
    assert len(FILES) >= 8


@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_oracle_reproduces_golden(oracle_mod, path):
    g = load(path)
    check(oracle_mod.OracleClay(int(g["k"]), int(g["m"]), int(g["d"])), g)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_gpu_reproduces_golden(path):
    from clay_amd import ClayCode
    g = load(path)
    check(ClayCode(int(g["k"]), int(g["m"]), int(g["d"])), g)

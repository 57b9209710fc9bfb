"""The host planner (symbolic replay of decode_layered / repair, clay_amd/csrc/plan.cpp)
checked on the CPU: its exported op DAG is executed with numpy (tests/plan_emu.py)
and compared byte-for-byte with the oracle -- including non-codeword inputs, so the
reference's RS row selection and iscore ordering are reproduced exactly."""
import itertools

import numpy as np
import pytest

from clay_amd import ClayCode
import plan_emu as E

CONFIGS = [(4, 2, 5), (6, 3, 8), (9, 3, 11), (10, 4, 13), (5, 3, 6), (7, 4, 9), (3, 3, 4),
           (8, 4, 11), (2, 4, 3)]


def _bufs(tn, a, sc):
    b = {i: np.zeros((a, sc), np.uint8) for i in range(tn)}
    b[2 * tn] = np.zeros((tn * a, sc), np.uint8)
    return b


@pytest.mark.parametrize("cfg", CONFIGS)
def test_plan_encode(oracle_mod, cfg):
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    tn, a = c.q * c.t, c.sub_chunk_no
    data = np.random.default_rng(k).integers(0, 256, k * a * 2 * 2 + 3, dtype=np.uint8)
    ref = o.encode_array(data)
    sc = ref.shape[1] // a
    bufs = _bufs(tn, a, sc)
    for i in range(k):
        bufs[i][:] = ref[i].reshape(a, sc)
    E.run_plan(c, E.export_plan(c, 0), bufs, sc)
    for p in range(m):
        assert np.array_equal(bufs[k + c.nu + p].reshape(-1), ref[k + p])


@pytest.mark.parametrize("cfg", CONFIGS)
def test_plan_decode_random_inputs(oracle_mod, cfg):
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    tn, a = c.q * c.t, c.sub_chunk_no
    rng = np.random.default_rng(100 + k)
    sc = 3
    chunk = a * sc
    pats = [list(e) for r in range(1, m + 1) for e in itertools.combinations(range(c.n), r)]
    rng.shuffle(pats)
    for er in pats[:10]:
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        av = {i: chunks[i] for i in range(c.n) if i not in er}
        ref = np.frombuffer(o.decode(av, er), np.uint8).reshape(k, chunk)
        mask = [0] * tn
        for e in er:
            mask[e if e < k else e + c.nu] = 1
        bufs = _bufs(tn, a, sc)
        for i in range(c.n):
            if i not in er:
                bufs[i if i < k else i + c.nu][:] = chunks[i].reshape(a, sc)
        E.run_plan(c, E.export_plan(c, 1, mask, mask), bufs, sc)
        for e in er:
            if e < k:
                assert np.array_equal(bufs[e].reshape(-1), ref[e]), (cfg, er, e)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_plan_repair_random_helpers(oracle_mod, cfg):
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    tn, a = c.q * c.t, c.sub_chunk_no
    rng = np.random.default_rng(200 + k)
    sc = 2
    for lost in range(c.n):
        info = o.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
        pd = {h: rng.integers(0, 256, len(idx) * sc, dtype=np.uint8) for h, idx in info}
        ref = np.frombuffer(o.repair(lost, pd, a * sc), np.uint8)
        hm = [0] * tn
        for h, _ in info:
            hm[h if h < k else h + c.nu] = 1
        bufs = {2 * tn: np.zeros((tn * a, sc), np.uint8), 2 * tn + 1: np.zeros((a, sc), np.uint8)}
        for h, _ in info:
            bufs[tn + (h if h < k else h + c.nu)] = pd[h].reshape(-1, sc)
        E.run_plan(c, E.export_plan(c, 2, hm, None, lost), bufs, sc)
        assert np.array_equal(bufs[2 * tn + 1].reshape(-1), ref), (cfg, lost)


def test_plan_stage_counts():
    """Launch counts the staged engine issues: encode of a q==m code is PRT -> RS -> PFT,
    with the PRT pairs over the data chunks folded into the RS rows (plan.cpp
    inline_inputs), so 2 dependent levels; 4 erasures in 4 y-sections of (10,4,13) need more."""
    c = ClayCode(10, 4, 13)
    assert len(E.export_plan(c, 0)[2]) - 1 == 2
    mask = [0] * 16
    for i in (0, 4, 8, 14):
        mask[i] = 1
    assert len(E.export_plan(c, 1, mask, mask)[2]) - 1 >= 5

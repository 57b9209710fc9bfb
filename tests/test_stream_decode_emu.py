"""CPU check of the streaming decodes' algebra (tests/stream_decode_emu.py) against the oracle:
the local kernel's step order (in-lane, g2-line and pair-inversion steps) for every local-eligible
pattern class, and the per-level rounds of the fused / split kernels, on random (non-codeword)
chunks, so only the reference's exact RS row choice and iscore order (decode.rs:167-408)
reproduce the bytes."""
import itertools

import numpy as np
import pytest

import stream_decode_emu as emu


def _patterns(n, pred, seed, n3, n4):
    pats = [list(e) for r in (1, 2) for e in itertools.combinations(range(n), r) if pred(list(e))]
    rng = np.random.default_rng(seed)
    for r, cnt in ((3, n3), (4, n4)):
        allp = [list(e) for e in itertools.combinations(range(n), r) if pred(list(e))]
        pats += [allp[i] for i in rng.permutation(len(allp))[:cnt]]
    return pats


def _check(oracle_mod, code, o, fn, er, sc, seed):
    chunks = np.random.default_rng(seed).integers(0, 256, (code.n, 256 * sc), dtype=np.uint8)
    got = fn(code, chunks, er)
    av = {i: chunks[i] for i in range(code.n) if i not in er}
    ref = np.frombuffer(o.decode(av, er), dtype=np.uint8).reshape(code.k, -1)
    for e in er:
        if e < code.k:
            assert np.array_equal(got[code.internal(e)].reshape(-1), ref[e]), (er, e)


def test_gf_tables_match_oracle(oracle_mod):
    for a, b in [(2, 2), (3, 7), (0x53, 0xCA), (255, 255), (1, 200), (0, 9)]:
        assert int(emu.MUL[a][b]) == oracle_mod.gf_mul(a, b)


@pytest.mark.parametrize("k", [10, 9])
def test_local_decode_algebra_matches_oracle(oracle_mod, k):
    code = emu.Code(oracle_mod, k)
    o = oracle_mod.OracleClay(k, 4, k + 3)
    pats = _patterns(code.n, lambda e: emu.local_eligible(code, e), k, 12, 12)
    for i, er in enumerate(pats):
        _check(oracle_mod, code, o, emu.local_decode, er, 2, 100 * k + i)
    # the verdict's patterns explicitly: {0}, {0,4}, {0,1}, {0,1,4}, {0,1,2,3}
    for er in ([0], [0, 4], [0, 1], [0, 1, 4], [0, 1, 2, 3]):
        assert emu.local_eligible(code, er)
        _check(oracle_mod, code, o, emu.local_decode, er, 3, 7 + len(er))


@pytest.mark.parametrize("k", [10, 9])
def test_fused_rounds_algebra_matches_oracle(oracle_mod, k):
    code = emu.Code(oracle_mod, k)
    o = oracle_mod.OracleClay(k, 4, k + 3)

    def one_per_section(er):
        secs = [code.internal(e) // 4 for e in er]
        return len(set(secs)) == len(secs)

    pats = _patterns(code.n, one_per_section, 3 * k, 6, 6)
    pats.insert(0, [0, 4, 8, 12] if k == 10 else [0, 4, 8, 11])
    for i, er in enumerate(pats[:20]):
        _check(oracle_mod, code, o, emu.fused_decode, er, 2, 300 * k + i)


@pytest.mark.parametrize("k", [10, 9])
def test_local256_phase_a_by_source_matches(oracle_mod, k):
    """k_stream_local256's section-G terms collected by source give the same presolved rows as
    the per-layer phase A, for every pattern with one erasure in its section plus at most one
    more, and every pair of erasures in one section."""
    code = emu.Code(oracle_mod, k)
    rng = np.random.default_rng(k)
    sc = 3
    pats = [[e] for e in range(code.n)] + [list(p) for p in itertools.combinations(range(code.n), 2)]
    n = 0
    for er in pats:
        per = [0] * 4
        for e in er:
            per[code.internal(e) // 4] += 1
        if not (max(per) == 1 or [n for n in per if n] == [2]):
            continue
        chunks = rng.integers(0, 256, (code.n, 256 * sc), dtype=np.uint8)
        C, E, used, rows, A = emu._setup(code, chunks, er)
        G = max(range(4), key=lambda y: (per[y], -y))
        want = emu._syndromes_presolved(code, C, E, used, rows)
        got = emu.presolved_by_source(code, C, E, used, rows, A, G)
        assert np.array_equal(got, want), er
        n += 1
    assert n > 50

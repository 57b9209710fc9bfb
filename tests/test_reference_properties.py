"""The reference's own unit and integration tests (src/lib.rs:261-778,
src/encode.rs:101-131, src/repair.rs:463-502, tests/integration.rs), re-run
against BOTH the oracle (CPU) and -- for everything that needs no GPU -- the
product's host logic (parameters, minimum_to_repair, input validation).

Byte-producing operations of the product run on the GPU and are covered by
tests/test_gpu_parity.py."""
import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode


def oc(oracle_mod, k, m, d):
    return oracle_mod.OracleClay(k, m, d)


def roundtrip(code, data, erasures):
    chunks = code.encode(data)
    av = {i: chunks[i] for i in range(len(chunks)) if i not in erasures}
    return code.decode(av, list(erasures))[:len(data)] == bytes(data)


# ---------------- lib.rs tests on the oracle ----------------
def test_basic_encode_decode(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    data = b"Test data for Clay codes - not empty!"
    chunks = c.encode(data)
    assert len(chunks) == 6
    assert c.decode({i: ch for i, ch in enumerate(chunks)}, [])[:len(data)] == data


def test_decode_with_erasures(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    data = b"Test data for Clay codes - testing erasure recovery!"
    for er in ([0], [5], [0, 5]):
        assert roundtrip(c, data, er)


def test_repair_correctness_and_bandwidth(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    data = b"Test data for repair correctness verification!!!!"
    chunks = c.encode(data)
    cs = len(chunks[0])
    sc = cs // c.sub_chunk_no
    for lost in range(c.n):
        info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
        pd = {h: b"".join(chunks[h][z * sc:(z + 1) * sc] for z in idx) for h, idx in info}
        assert c.repair(lost, pd, cs) == chunks[lost]
        assert sum(len(v) for v in pd.values()) < c.k * cs * 7 // 10


@pytest.mark.parametrize("k,m,d", [(4, 2, 5), (9, 3, 11), (10, 4, 13)])
def test_various_parameters(oracle_mod, k, m, d):
    c = oc(oracle_mod, k, m, d)
    data = bytes(i % 256 for i in range(k * c.sub_chunk_no * 2))
    assert roundtrip(c, data, [0])


@pytest.mark.parametrize("k,m,d", [(4, 2, 5), (9, 3, 11)])
def test_repair_all_nodes_various_params(oracle_mod, k, m, d):
    c = oc(oracle_mod, k, m, d)
    data = bytes((i * 7 + 13) % 256 for i in range(k * c.sub_chunk_no))
    chunks = c.encode(data)
    cs = len(chunks[0])
    sc = cs // c.sub_chunk_no
    for lost in range(c.n):
        info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
        pd = {h: b"".join(chunks[h][z * sc:(z + 1) * sc] for z in idx) for h, idx in info}
        assert c.repair(lost, pd, cs) == chunks[lost]


def test_decode_max_erasures(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    data = bytes(range(256))
    for er in ([0, 5], [0, 1], [4, 5], [1, 3]):
        assert roundtrip(c, data, er)


def test_random_data(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    data = np.random.default_rng(99).integers(0, 256, c.k * c.sub_chunk_no * 4, dtype=np.uint8).tobytes()
    assert roundtrip(c, data, []) and roundtrip(c, data, [2])


# ---------------- tests/integration.rs on the oracle ----------------
def test_full_repair_flow_with_bandwidth_check(oracle_mod):
    c = oc(oracle_mod, 10, 4, 13)
    assert (c.n, c.k, c.m, c.d, c.q, c.sub_chunk_no, c.beta) == (14, 10, 4, 13, 4, 256, 64)
    data = bytes((i * 17 + 31) % 256 for i in range(c.k * c.sub_chunk_no))
    chunks = c.encode(data)
    assert len(chunks) == 14
    cs = len(chunks[0])
    sc = cs // c.sub_chunk_no
    info = c.minimum_to_repair(0, list(range(1, c.n)))
    assert len(info) == c.d
    rb = sum(len(idx) * sc for _, idx in info)
    assert rb / (c.k * cs) < 0.35
    pd = {h: b"".join(chunks[h][z * sc:(z + 1) * sc] for z in idx) for h, idx in info}
    assert c.repair(0, pd, cs) == chunks[0]


def test_multi_erasure_decode(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    data = bytes(i % 256 for i in range(512))
    for er in ([0], [5], [0, 5], [0, 1], [4, 5], [1, 3]):
        assert roundtrip(c, data, er)


@pytest.mark.parametrize("k,m,d", [(4, 2, 5), (9, 3, 11), (10, 4, 13)])
def test_repair_bandwidth_advantage(oracle_mod, k, m, d):
    c = oc(oracle_mod, k, m, d)
    data = bytes(i % 256 for i in range(k * c.sub_chunk_no))
    cs = len(c.encode(data)[0])
    sc = cs // c.sub_chunk_no
    for lost in range(c.n):
        info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
        assert sum(len(idx) * sc for _, idx in info) < k * cs


# ---------------- encode.rs tests ----------------
def test_encode_chunk_count_empty_and_alignment(oracle_mod):
    c = oc(oracle_mod, 4, 2, 5)
    assert len(c.encode(b"Test data for encoding")) == c.n
    chunks = c.encode(b"")
    assert len(chunks) == c.n and len({len(x) for x in chunks}) == 1
    for ch in c.encode(bytes([0xAB] * 100)):
        assert len(ch) % c.sub_chunk_no == 0


# ---------------- product host logic == reference (no GPU needed) ----------------
@pytest.mark.parametrize("k,m,d", [(4, 2, 5), (9, 3, 11), (10, 4, 13), (6, 3, 8), (5, 3, 6),
                                   (1, 2, 2), (20, 4, 23)])
def test_product_parameters_match(oracle_mod, k, m, d):
    a, b = ClayCode(k, m, d), oc(oracle_mod, k, m, d)
    for f in ("k", "m", "n", "d", "q", "t", "nu", "sub_chunk_no", "beta"):
        assert getattr(a, f) == getattr(b, f), f
    assert a.normalized_repair_bandwidth() == pytest.approx(b.normalized_repair_bandwidth())
    for n in (0, 1, 100, 12345, 1 << 20):
        assert a.encoded_chunk_size(n) == b.encoded_chunk_size(n)


def test_product_normalized_repair_bandwidth():
    for (k, m, d), exp in [((4, 2, 5), 0.625), ((9, 3, 11), 0.407), ((10, 4, 13), 0.325)]:
        assert abs(ClayCode(k, m, d).normalized_repair_bandwidth() - exp) < 0.01


def test_product_new_default_and_invalid():
    a, b = ClayCode.new_default(4, 2), ClayCode(4, 2, 5)
    assert (a.d, a.q, a.t, a.sub_chunk_no, a.beta) == (b.d, b.q, b.t, b.sub_chunk_no, b.beta)
    assert ClayCode.new_default(10, 4).d == 13
    for args in ((0, 2, 1), (4, 0, 3), (4, 2, 4), (4, 2, 6)):
        with pytest.raises(clay_amd.InvalidParameters):
            ClayCode(*args)


def test_product_overflow_variant(oracle_mod):
    # q = 2, n + nu = 130 -> t = 65 -> 2^65 overflows usize
    with pytest.raises(clay_amd.Overflow) as e:
        ClayCode(127, 3, 128)
    with pytest.raises(oracle_mod.OracleError) as o:
        oc(oracle_mod, 127, 3, 128)
    assert str(e.value) == o.value.msg


@pytest.mark.parametrize("k,m,d", [(4, 2, 5), (9, 3, 11), (10, 4, 13), (6, 3, 8), (5, 3, 6)])
def test_product_minimum_to_repair_matches(oracle_mod, k, m, d):
    a, b = ClayCode(k, m, d), oc(oracle_mod, k, m, d)
    rng = np.random.default_rng(k * 100 + m)
    for lost in range(a.n):
        for trial in range(4):
            av = [i for i in range(a.n + 2) if i != lost]  # out-of-range extras are not validated
            rng.shuffle(av)
            av = av[:a.d + trial - 1]
            try:
                exp = b.minimum_to_repair(lost, av)
            except oracle_mod.OracleError as oe:
                with pytest.raises(clay_amd.ClayError) as pe:
                    a.minimum_to_repair(lost, av)
                assert pe.value.kind == oe.kind and str(pe.value) == oe.msg
                continue
            assert a.minimum_to_repair(lost, av) == exp
    with pytest.raises(clay_amd.InvalidParameters):
        a.minimum_to_repair(a.n, [0])


def _decode_error_cases(code):
    ch = [bytes(code.sub_chunk_no * 2)] * code.n
    yield {}, [0]                                                   # empty available
    yield {i: ch[i] for i in range(code.m + 1, code.n)}, list(range(code.m + 1))  # too many
    yield {i: bytes(3) for i in range(1, code.n)}, [0]             # bad chunk size
    bad = {i: ch[i] for i in range(1, code.n)}
    bad[code.n - 1] = ch[0] + b"\0"
    yield bad, [0]                                                  # inconsistent sizes
    yield {**{i: ch[i] for i in range(code.n)}, 100: ch[0]}, []     # index out of range
    yield {i: ch[i] for i in range(1, code.n)}, [100]               # erasure out of range
    yield {i: ch[i] for i in range(code.n)}, [0]                    # overlap -> "both"
    yield {i: ch[i] for i in range(2, code.n)}, [0]                 # wrong count -> "Expected"
    yield {i: ch[i] for i in range(1, code.n) if i != 2}, [0, 0]    # neither erased nor provided


@pytest.mark.parametrize("k,m,d", [(4, 2, 5), (10, 4, 13)])
def test_product_decode_validation_matches(oracle_mod, k, m, d):
    """Validation runs on the host before any GPU work: identical kind, payload, message."""
    a, b = ClayCode(k, m, d), oc(oracle_mod, k, m, d)
    for av, er in _decode_error_cases(a):
        with pytest.raises(oracle_mod.OracleError) as oe:
            b.decode(av, er)
        with pytest.raises(clay_amd.ClayError) as pe:
            a.decode(av, er)
        assert pe.value.kind == oe.value.kind, (av.keys(), er)
        assert pe.value.fields == oe.value.fields and str(pe.value) == oe.value.msg
    assert a.decode({}, []) == b"" == b.decode({}, [])


def test_product_repair_validation_matches(oracle_mod):
    a, b = ClayCode(10, 4, 13), oc(oracle_mod, 10, 4, 13)
    sc = 2
    good = {h: bytes(64 * sc) for h in range(1, 14)}
    cases = [
        (14, good, 512),                                  # lost out of range
        (0, {h: good[h] for h in range(1, 12)}, 512),     # insufficient helpers
        (0, good, 0), (0, good, 511),                     # chunk size
        (0, {h: good[h] for h in range(4, 14)} | {1: good[1], 2: good[2], 99: bytes(128)}, 512),  # missing y-section peer 3
        (0, {**{h: good[h] for h in range(1, 14)}, 20: bytes(128)}, 512),      # helper index range
        (0, {**{h: good[h] for h in range(1, 13)}, 13: bytes(127)}, 512),      # helper data size
    ]
    for lost, hd, cs in cases:
        with pytest.raises(oracle_mod.OracleError) as oe:
            b.repair(lost, hd, cs)
        with pytest.raises(clay_amd.ClayError) as pe:
            a.repair(lost, hd, cs)
        assert pe.value.kind == oe.value.kind and pe.value.fields == oe.value.fields
        assert str(pe.value) == oe.value.msg


def test_product_decode_rs_shard_limit_matches(oracle_mod):
    """(1,256,256): q = 256, original_count + recovery_count = 512 > 256.  decode_layered
    builds ReedSolomon::new before any layer work (decode.rs:175-180), so even a decode with
    no data node erased fails with ReconstructionFailed("RS init failed: TooManyShards")."""
    a, b = ClayCode(1, 256, 256), oc(oracle_mod, 1, 256, 256)
    chunk = a.sub_chunk_no  # 65,536: the smallest valid chunk
    av = {i: bytes(chunk) for i in range(1, a.n)}
    for er in ([0], []):
        avail = av if er else {**av, 0: bytes(chunk)}
        with pytest.raises(oracle_mod.OracleError) as oe:
            b.decode(avail, er)
        with pytest.raises(clay_amd.ClayError) as pe:
            a.decode(avail, er)
        assert pe.value.kind == oe.value.kind and str(pe.value) == oe.value.msg

"""GPU parity of the streaming decodes (stream_decode.hpp phase A + the local decode,
stream_local.hpp, and the fused decode v2, stream_fused2.hpp) against the oracle.

The kernels serve q = 4, t = 4 codes ((10,4,13) and (9,4,12)) in the "stream" executor mode: the
local decode for erasures in one y-section plus at most one other, the fused decode v2 for 2-4
erasures in distinct y-sections (decode.rs:167-257 with the reference's iscore order).  Inputs are random, i.e. NOT codewords: only the reference's exact RS row
choice (reconstruct from the first k+nu present shards, decode.rs:374) reproduces those bytes,
so these tests pin the syndrome formulation's "used" / "ignored" shard handling as well."""
import itertools

import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode

pytestmark = pytest.mark.gpu


def _internal(c, e):
    return e if e < c.k else e + c.nu


def stream_eligible(c, er):
    per = [0] * c.t
    for e in er:
        per[_internal(c, e) // c.q] += 1
    return len(er) >= 1 and max(per) <= 1


def _patterns(c, seed, n3, n4):
    pats = [list(e) for r in (1, 2) for e in itertools.combinations(range(c.n), r)]
    rng = np.random.default_rng(seed)
    for r, cnt in ((3, n3), (4, n4)):
        allp = [list(e) for e in itertools.combinations(range(c.n), r)]
        for i in rng.permutation(len(allp))[:cnt]:
            pats.append(allp[i])
    return pats


def local_eligible(c, er):
    """k_stream_local: erasures in one y-section plus at most one erasure in one other section."""
    per = [0] * c.t
    for e in er:
        per[_internal(c, e) // c.q] += 1
    busy = [n for n in per if n]
    return len(busy) == 1 or (len(busy) == 2 and min(busy) == 1)


def stream_path(c, er):
    """The kernel exec mode "stream" runs a pattern on (None: the plan executor)."""
    per = sorted((sum(1 for e in er if _internal(c, e) // c.q == y) for y in range(c.t)), reverse=True)
    if len(er) == 3 and per[:2] == [2, 1] and fused2_eligible(c, er, two=True):
        return "stream-fused2"  # (2,1) sections: the fused decode v2 first (round 6)
    if local_eligible(c, er):
        per = [0] * c.t
        for e in er:
            per[_internal(c, e) // c.q] += 1
        return "stream-local256" if max(per) == 1 or [n for n in per if n] == [2] else "stream-local"
    if fused2_eligible(c, er, two=True):
        return "stream-fused2"
    return None


@pytest.fixture
def stream_mode():
    prev = clay_amd.set_exec_mode("stream")
    yield
    clay_amd.set_exec_mode(prev)


def _decode_dev(torch, c, chunks, er, chunk, want_parity=True):
    full = torch.from_numpy(chunks).cuda()
    outs = torch.full((c.n, chunk), 0xA5, dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(c.n)], er,
                    [outs[i] if i in er and (i < c.k or want_parity) else None for i in range(c.n)], chunk)
    torch.cuda.synchronize()
    return outs.cpu().numpy()


def _oracle_erased(o, c, chunks, er):
    """Oracle C of every erased node (data via decode; parity via re-encode of the decoded data,
    which equals the reference's U -> C of the parity node only for codewords -- so parity
    outputs are checked on codewords, data outputs on random inputs)."""
    av = {i: chunks[i] for i in range(c.n) if i not in er}
    data = np.frombuffer(o.decode(av, er), dtype=np.uint8).reshape(c.k, -1)
    return data


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [512, 520, 64 * 37 + 40])
def test_stream_decode_patterns_random_inputs(oracle_mod, torch_cuda, stream_mode, cfg, sc):
    """Every 1- and 2-erasure pattern and a sample of 3- and 4-erasure patterns on random
    (non-codeword) chunks: the erased data chunks match the oracle bit for bit; a streaming
    kernel ran for every eligible pattern (the rest fall back to the plan executor)."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + cfg[0])
    n_stream = 0
    for er in _patterns(c, sc, 24, 40):
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        got = _decode_dev(torch, c, chunks, er, chunk, want_parity=False)
        path = clay_amd.last_exec_path()
        if stream_path(c, er):
            assert path == stream_path(c, er), (er, path)
            n_stream += 1
        ref = _oracle_erased(o, c, chunks, er)
        for e in er:
            if e < c.k:
                assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e, path)
            else:
                assert np.all(got[e] == 0xA5), "parity output written though not requested"
    assert n_stream > 0


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [520, 64 * 8 * 33 + 24])
def test_stream_decode_codeword_incl_parity(oracle_mod, torch_cuda, stream_mode, cfg, sc):
    """Codewords with data AND parity erased: every rebuilt chunk (parity included) equals the
    encoded one; patterns with up to 4 erasures, one per y-section (the BASELINE worst case
    {0,4,8,12} first)."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(sc).integers(0, 256, c.k * chunk, dtype=np.uint8))
    pats = [[0, 4, 8, 12]] if cfg == (10, 4, 13) else [[0, 4, 8, 11]]
    pats += [p for p in _patterns(c, 5, 12, 12) if stream_path(c, p)]
    for er in pats:
        got = _decode_dev(torch, c, ref, er, chunk)
        assert clay_amd.last_exec_path() == stream_path(c, er), er
        for e in er:
            assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e)


def test_stream_decode_matches_grouped_executor(oracle_mod, torch_cuda, stream_mode):
    """Same random inputs through the streaming kernel and the grouped plan executor: identical
    bytes, including the rebuilt parity chunk."""
    torch = torch_cuda
    c = ClayCode(10, 4, 13)
    sc = 64 * 50 + 8
    chunk = c.sub_chunk_no * sc
    chunks = np.random.default_rng(9).integers(0, 256, (c.n, chunk), dtype=np.uint8)
    er = [1, 6, 9, 13]
    a = _decode_dev(torch, c, chunks, er, chunk)
    assert clay_amd.last_exec_path() == "stream-fused2"
    clay_amd.set_exec_mode("grouped")
    b = _decode_dev(torch, c, chunks, er, chunk)
    assert clay_amd.last_exec_path() == "grouped"
    clay_amd.set_exec_mode("stream")
    for e in er:
        assert np.array_equal(a[e], b[e]), e


def f2_fits(c, er, two=False):
    """The host's round-capacity check (engine.hip f2_plan): per section Y with an erasure and
    iscore level L, P(Y, L) = passes of 64 lanes x 8-byte pieces over the layers with z_Y in E_Y
    and L erased sections red; the four loader waves: at least one per section with an erasure,
    split to minimise the sum over levels of the busiest wave's passes; a wave holds <= kF2Iters
    (two) / kF2Iters1 passes per level."""
    iters = [5, 4, 2, 1] if two else [6, 4, 2, 1]
    em = [0] * c.t
    for e in er:
        i = _internal(c, e)
        em[i // c.q] |= 1 << (i % c.q)
    P = {}
    for Y in range(c.t):
        if not em[Y]:
            continue
        for L in range(1, 5):
            n = 0
            for z in range(256):
                d = [(z >> (2 * (3 - y))) & 3 for y in range(4)]
                red = sum(1 for y in range(4) if (em[y] >> d[y]) & 1)
                n += 1 if (em[Y] >> d[Y]) & 1 and red == L else 0
            P[Y, L] = (n * 8 + 63) // 64
    act = [y for y in range(c.t) if em[y]]
    best, bcost = None, None
    for n in itertools.product(range(5), repeat=4):  # lexicographic, as the host's loops
        if sum(n) != 4 or any((n[y] > 0) != (y in act) for y in range(4)):
            continue
        mx = [max(-(-P[y, L] // n[y]) for y in act) for L in range(1, 5)]
        if any(m > iters[L] for L, m in enumerate(mx)):
            continue
        cost = sum(mx)
        if bcost is None or cost < bcost:
            best, bcost = n, cost
    return best is not None


def fused2_eligible(c, er, two=False):
    """k_stream_fused2: 2-4 erasures in distinct y-sections (two=True: at most two per section,
    round 6) whose round targets fit the kernel's item registers, and a ring of 10 - e node buffers
    that holds any two neighbouring sections' surviving real nodes."""
    per = [0] * c.t
    for e in er:
        per[_internal(c, e) // c.q] += 1
    if not 2 <= len(er) <= c.t or max(per) > (2 if two else 1) or not f2_fits(c, er, two):
        return False
    alive = [0] * c.t
    for i in range(c.n):
        if i not in er:
            alive[_internal(c, i) // c.q] += 1
    rb = 10 - len(er)
    if two:  # round 6: neighbouring sections beyond the ring run as split steps
        return max(alive) <= rb
    return all(alive[y] + alive[(y + 1) % c.t] <= rb for y in range(c.t))  # incl. section 3 -> next tile's 0


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [512, 520, 64 * 37 + 40])
def test_fused2_decode_random_inputs(oracle_mod, torch_cuda, cfg, sc):
    """Exec mode "stream-fused2" (stream_fused2.hpp): samples of the eligible 4-, 3- and 2-erasure
    patterns (distinct sections; the unused survivor of a 2- or 3-erasure pattern may share a
    section with an erasure) on random chunks, erased data chunks bit-exact vs the oracle."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + 3 * cfg[0])
    pats = []
    for r, cnt in ((4, 30), (3, 20), (2, 10)):
        allp = [list(e) for e in itertools.combinations(range(c.n), r) if fused2_eligible(c, list(e))]
        pats += [allp[i] for i in rng.permutation(len(allp))[:cnt]]
    pats.insert(0, [0, 4, 8, 12] if cfg == (10, 4, 13) else [0, 4, 8, 11])
    pats.insert(1, [0, 4, 8])
    pats.insert(2, [4, c.n - 1])
    prev = clay_amd.set_exec_mode("stream-fused2")
    try:
        for er in pats:
            chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
            got = _decode_dev(torch, c, chunks, er, chunk, want_parity=False)
            assert clay_amd.last_exec_path() == "stream-fused2", (er, clay_amd.last_exec_path())
            ref = _oracle_erased(o, c, chunks, er)
            for e in er:
                if e < c.k:
                    assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e)
    finally:
        clay_amd.set_exec_mode(prev)


@pytest.mark.parametrize("sc", [520, 64 * 8 * 33 + 24])
def test_fused2_decode_codeword_incl_parity_and_grouped(oracle_mod, torch_cuda, sc):
    """The BASELINE worst case {0,4,8,12} and 3- / 2-erasure patterns with parity nodes on a
    codeword (every rebuilt chunk incl. parity) and on random inputs against the grouped plan
    executor (parity outputs included)."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(sc).integers(0, 256, c.k * chunk, dtype=np.uint8))
    prev = clay_amd.set_exec_mode("stream-fused2")
    try:
        for er in ([0, 4, 8, 12], [0, 4, 8], [1, 9, 13], [5, 12]):
            clay_amd.set_exec_mode("stream-fused2")
            got = _decode_dev(torch, c, ref, er, chunk)
            assert clay_amd.last_exec_path() == "stream-fused2", er
            for e in er:
                assert np.array_equal(got[e], ref[e]), (er, e)
            chunks = np.random.default_rng(sc + len(er)).integers(0, 256, (c.n, chunk), dtype=np.uint8)
            a = _decode_dev(torch, c, chunks, er, chunk)
            clay_amd.set_exec_mode("grouped")
            b = _decode_dev(torch, c, chunks, er, chunk)
            assert clay_amd.last_exec_path() == "grouped"
            for e in er:
                assert np.array_equal(a[e], b[e]), (er, e)
    finally:
        clay_amd.set_exec_mode(prev)


def _two_in_a_section(c, r=4):
    """The 4-erasure patterns with two erasures in a section and the others elsewhere ((2,1,1) and
    (2,2) sections), which round 6 moved from the grouped executor to k_stream_fused2."""
    out = []
    for er in itertools.combinations(range(c.n), r):
        per = [0] * c.t
        for e in er:
            per[_internal(c, e) // c.q] += 1
        if max(per) == 2 and not local_eligible(c, list(er)) and fused2_eligible(c, list(er), two=True):
            out.append(list(er))
    return out


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [512, 520, 64 * 37 + 40])
def test_fused2_two_erasures_in_a_section_random_inputs(oracle_mod, torch_cuda, cfg, sc):
    """Auto mode on 4-erasure patterns with two erasures in one y-section ((2,1,1): {0,1,4,8},
    {8,9,0,4}; (2,2): {0,1,4,5}; with parity nodes: {0,1,4,12}) and a random sample of the rest:
    k_stream_fused2 runs (the both-erased PFT pairs inverted after the rounds), erased data chunks
    bit-exact vs the oracle on random (non-codeword) chunks, ragged and sc % 16 == 8 tiles."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc * 7 + cfg[0])
    allp = _two_in_a_section(c)
    assert len(allp) == (750 if cfg == (10, 4, 13) else 540)
    pats = [p for p in ([0, 1, 4, 8], [8, 9, 0, 4], [0, 1, 4, 5], [0, 1, 4, 12], [4, 5, 12, 13], [0, 8, 9, 10])
            if sorted(p) in allp]
    pats += [allp[i] for i in rng.permutation(len(allp))[:14]]
    for er in pats:
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        got = _decode_dev(torch, c, chunks, er, chunk, want_parity=False)
        assert clay_amd.last_exec_path() == "stream-fused2", (er, clay_amd.last_exec_path())
        ref = _oracle_erased(o, c, chunks, er)
        for e in er:
            if e < c.k:
                assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e)


@pytest.mark.parametrize("sc", [520, 64 * 8 * 33 + 24])
def test_fused2_two_erasures_in_a_section_codeword_and_grouped(oracle_mod, torch_cuda, sc):
    """(2,1,1) / (2,2) patterns incl. parity nodes on a codeword (every rebuilt chunk, parity
    included, equals the encoded one) and on random chunks against the grouped plan executor
    (parity outputs included)."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(sc).integers(0, 256, c.k * chunk, dtype=np.uint8))
    for er in ([0, 1, 4, 12], [12, 13, 0, 4], [12, 13, 1, 2], [8, 9, 12, 13], [2, 3, 6, 13]):
        got = _decode_dev(torch, c, ref, er, chunk)
        assert clay_amd.last_exec_path() == "stream-fused2", er
        for e in er:
            assert np.array_equal(got[e], ref[e]), (er, e)
        chunks = np.random.default_rng(sc + er[0]).integers(0, 256, (c.n, chunk), dtype=np.uint8)
        a = _decode_dev(torch, c, chunks, er, chunk)
        prev = clay_amd.set_exec_mode("grouped")
        try:
            b = _decode_dev(torch, c, chunks, er, chunk)
        finally:
            clay_amd.set_exec_mode(prev)
        for e in er:
            assert np.array_equal(a[e], b[e]), (er, e)


@pytest.mark.slow
@pytest.mark.parametrize("er", [[0, 1, 4, 8], [0, 1, 4, 5], [8, 9, 0, 4], [0, 1, 4, 12]])
def test_two_in_a_section_1GiB(oracle_mod, torch_cuda, er):
    """(2,1,1) / (2,2) patterns at the BASELINE stripe (sc 419,432) under auto (k_stream_fused2,
    TWO): on random chunks, column slices of every erased data chunk match the oracle's decode of
    the same slices (positions [p0, p0 + 64) of every sub-chunk are an independent instance); on a
    codeword (the product encode) every erased chunk, parity included, comes back."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    chunk = c.encoded_chunk_size(1 << 30)
    sc = chunk // c.sub_chunk_no
    g = torch.Generator(device="cuda")
    g.manual_seed(sum(er))
    full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda", generator=g)
    outs = torch.zeros((c.n, chunk), dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(c.n)], er,
                    [outs[i] if i in er and i < c.k else None for i in range(c.n)], chunk)
    torch.cuda.synchronize()
    assert clay_amd.last_exec_path() == "stream-fused2"
    for p0 in (0, sc // 2 + 8, sc - 64):
        s = full[:, :].view(c.n, c.sub_chunk_no, sc)[:, :, p0:p0 + 64].cpu().numpy().reshape(c.n, -1)
        got = outs.view(c.n, c.sub_chunk_no, sc)[:, :, p0:p0 + 64].cpu().numpy().reshape(c.n, -1)
        ref = np.frombuffer(o.decode({i: s[i] for i in range(c.n) if i not in er}, er), np.uint8).reshape(c.k, -1)
        for e in er:
            if e < c.k:
                assert np.array_equal(got[e], ref[e]), (er, p0, e)
    # codeword: the product encode (oracle-checked by the encode tests), then decode
    c.encode_device([full[i] for i in range(c.k)], [full[c.k + x] for x in range(c.m)], chunk)
    outs.zero_()
    c.decode_device([None if i in er else full[i] for i in range(c.n)], er,
                    [outs[i] if i in er else None for i in range(c.n)], chunk)
    torch.cuda.synchronize()
    assert clay_amd.last_exec_path() == "stream-fused2"
    for e in er:
        assert torch.equal(outs[e], full[e]), (er, e)


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [520, 64 * 37 + 40])
def test_fused2_two_erasures_small_patterns(oracle_mod, torch_cuda, cfg, sc):
    """Exec mode "stream-fused2" on 2- and 3-erasure patterns with two erasures in a section
    ((2) and (2,1) sections: the loader-wave plan gives the busy section 3-4 waves), random
    chunks, erased data chunks bit-exact vs the oracle."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + cfg[0])
    pats = [[0, 1], [2, 3], [0, 1, 4], [0, 4, 5], [c.n - 2, c.n - 1, 0], [c.n - 1, 1, 2]]
    prev = clay_amd.set_exec_mode("stream-fused2")
    try:
        for er in pats:
            assert fused2_eligible(c, er, two=True), er
            chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
            got = _decode_dev(torch, c, chunks, er, chunk, want_parity=False)
            assert clay_amd.last_exec_path() == "stream-fused2", (er, clay_amd.last_exec_path())
            ref = _oracle_erased(o, c, chunks, er)
            for e in er:
                if e < c.k:
                    assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e)
    finally:
        clay_amd.set_exec_mode(prev)

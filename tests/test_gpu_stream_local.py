"""GPU parity of the local streaming decodes (exec mode "stream-local" and auto) against the
oracle: k_stream_local256 (stream_local256.hpp, 256-byte row runs) for one erasure in a section
plus at most one in another, k_stream_local (stream_local.hpp, 64-byte tiles) for the rest.

The kernel serves q = 4, t = 4 codes ((10,4,13), (9,4,12)) whose erasures lie in one y-section
plus at most one erasure in one other section: single erasures, two erasures in two sections
({0,4}), same-section patterns whose PFT pairs are both erased ({0,1}, {0,1,2,3}: the
get_coupled_from_uncoupled branch, decode.rs:228-232) and mixes ({0,1,4}).  Inputs are random
(NOT codewords), so only the reference's exact RS row choice (reconstruct from the first k+nu
present shards, decode.rs:374) and iscore order reproduce the bytes."""
import itertools

import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode

pytestmark = pytest.mark.gpu


def _internal(c, e):
    return e if e < c.k else e + c.nu


def local_eligible(c, er):
    per = [0] * c.t
    for e in er:
        per[_internal(c, e) // c.q] += 1
    nz = sorted([p for p in per if p], reverse=True)
    return 1 <= len(er) <= c.m and len(nz) <= 2 and (len(nz) < 2 or nz[1] == 1)


def local_path(c, er, mode="stream-local"):
    """The kernel a local-eligible pattern runs on (8-byte rows, sc >= 512): in auto, the (2,1)
    patterns take the fused decode v2 first (round 6; every one of them fits it for (10,4,13) and
    (9,4,12), tests/test_gpu_stream_decode.py::fused2_eligible)."""
    per = [0] * c.t
    for e in er:
        per[_internal(c, e) // c.q] += 1
    busy = [n for n in per if n]
    if mode == "auto" and len(er) == 3 and sorted(busy) == [1, 2]:
        return "stream-fused2"
    return "stream-local256" if max(per) == 1 or busy == [2] else "stream-local"


def _local_patterns(c, seed, n3, n4):
    pats = [list(e) for r in (1, 2) for e in itertools.combinations(range(c.n), r)]
    rng = np.random.default_rng(seed)
    for r, cnt in ((3, n3), (4, n4)):
        allp = [list(e) for e in itertools.combinations(range(c.n), r) if local_eligible(c, list(e))]
        for i in rng.permutation(len(allp))[:cnt]:
            pats.append(allp[i])
    return pats


@pytest.fixture(params=["stream-local", "auto"])
def local_mode(request):
    prev = clay_amd.set_exec_mode(request.param)
    yield request.param
    clay_amd.set_exec_mode(prev)


def _decode_dev(torch, c, chunks, er, chunk, want_parity=True):
    full = torch.from_numpy(chunks).cuda()
    outs = torch.full((c.n, chunk), 0xA5, dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(c.n)], er,
                    [outs[i] if i in er and (i < c.k or want_parity) else None for i in range(c.n)], chunk)
    torch.cuda.synchronize()
    return outs.cpu().numpy()


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [512, 520, 64 * 37 + 40])
def test_local_decode_random_inputs(oracle_mod, torch_cuda, local_mode, cfg, sc):
    """Every 1- and 2-erasure pattern and samples of the eligible 3- and 4-erasure patterns on
    random chunks: the erased data chunks equal the oracle's bit for bit, the local kernel ran
    for every eligible pattern, and unrequested parity outputs stay untouched."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + 7 * cfg[0])
    n_local = 0
    for er in _local_patterns(c, sc, 16, 16):
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        got = _decode_dev(torch, c, chunks, er, chunk, want_parity=False)
        path = clay_amd.last_exec_path()
        if local_eligible(c, er):
            assert path == local_path(c, er, local_mode), (er, path)
            n_local += 1
        av = {i: chunks[i] for i in range(c.n) if i not in er}
        ref = np.frombuffer(o.decode(av, er), dtype=np.uint8).reshape(c.k, -1)
        for e in er:
            if e < c.k:
                assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e, path)
            else:
                assert np.all(got[e] == 0xA5), "parity output written though not requested"
    assert n_local > 0


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [520, 64 * 8 * 33 + 24])
def test_local_decode_codeword_incl_parity(oracle_mod, torch_cuda, local_mode, cfg, sc):
    """Codewords with data AND parity erased: every rebuilt chunk (parity included) equals the
    encoded one, for the verdict's patterns and samples of every eligible size."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(sc).integers(0, 256, c.k * chunk, dtype=np.uint8))
    pats = [[0], [0, 4], [0, 1], [0, 1, 4], [0, 1, 2, 3], [c.n - 1], [c.n - 2, c.n - 1], [0, c.n - 1]]
    pats += [p for p in _local_patterns(c, 3, 10, 10) if local_eligible(c, p)][::5]
    for er in pats:
        assert local_eligible(c, er), er
        got = _decode_dev(torch, c, ref, er, chunk)
        assert clay_amd.last_exec_path() == local_path(c, er, local_mode), er
        for e in er:
            assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e)


@pytest.mark.parametrize("er", [[0], [0, 4], [0, 1], [0, 1, 4], [0, 1, 2, 3], [2, 13], [8, 9, 12], [10, 11, 12, 13]])
def test_local_decode_matches_grouped_incl_parity(oracle_mod, torch_cuda, er):
    """Random (non-codeword) inputs through the local kernel and the grouped plan executor:
    identical bytes for every erased node, the rebuilt parity chunks included (the oracle's decode
    returns data only)."""
    torch = torch_cuda
    c = ClayCode(10, 4, 13)
    sc = 64 * 50 + 8
    chunk = c.sub_chunk_no * sc
    chunks = np.random.default_rng(len(er) * 31 + er[0]).integers(0, 256, (c.n, chunk), dtype=np.uint8)
    prev = clay_amd.set_exec_mode("stream-local")
    try:
        a = _decode_dev(torch, c, chunks, er, chunk)
        assert clay_amd.last_exec_path() == local_path(c, er)
        clay_amd.set_exec_mode("grouped")
        b = _decode_dev(torch, c, chunks, er, chunk)
        assert clay_amd.last_exec_path() == "grouped"
    finally:
        clay_amd.set_exec_mode(prev)
    for e in er:
        assert np.array_equal(a[e], b[e]), e


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("sc", [513, 515, 1037, 64 * 37 + 42])
def test_local256_any_subchunk(oracle_mod, torch_cuda, cfg, sc):
    """k_stream_local256 at sub-chunks that are not multiples of 8 (rows at odd byte offsets:
    the (9,4,12) 1 GiB stripe has sc = 2 mod 8), for every 1-erasure pattern and the 2-erasure
    patterns it takes, on random chunks vs the oracle; the other local patterns fall back to the
    plan executors there (the 64-byte kernel needs 8-byte rows)."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc * 3 + cfg[0])
    pats = [[e] for e in range(c.n)] + [list(p) for p in itertools.combinations(range(c.n), 2)][::3]
    pats += [[0, 1, 4]]
    n256 = 0
    for er in pats:
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        got = _decode_dev(torch, c, chunks, er, chunk, want_parity=False)
        path = clay_amd.last_exec_path()
        if local_eligible(c, er) and local_path(c, er) == "stream-local256":
            assert path == "stream-local256", (er, path)
            n256 += 1
        else:
            assert not path.startswith("stream-local"), (er, path)
        av = {i: chunks[i] for i in range(c.n) if i not in er}
        ref = np.frombuffer(o.decode(av, er), dtype=np.uint8).reshape(c.k, -1)
        for e in er:
            if e < c.k:
                assert np.array_equal(got[e], ref[e]), (cfg, sc, er, e, path)
            else:
                assert np.all(got[e] == 0xA5), "parity output written though not requested"
    assert n256 > 10


@pytest.mark.parametrize("sc", [512, 64 * 37 + 40])
def test_local256_misaligned_chunk_pointers(oracle_mod, torch_cuda, sc):
    """sc % 8 == 0 but chunk pointers offset 1-7 bytes from 8-byte alignment (slices of one
    larger buffer): the ANY instantiation of k_stream_local256 runs (its full-tile DMA and the
    16-byte stores at odd addresses), full and partial tiles, inputs and outputs misaligned by
    different amounts; bytes vs the oracle, neighbouring bytes of the outputs untouched
    (ADVICE r05)."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + 99)
    for k, er in enumerate(([0], [5], [12], [0, 4], [3, 13], [0, 1])):
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        pitch = chunk + 64
        src = torch.zeros(c.n * pitch + 64, dtype=torch.uint8, device="cuda")
        dst = torch.full((c.n * pitch + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        ins, ous = [], []
        for i in range(c.n):
            a = i * pitch + 1 + (i + k) % 7       # 1..7 bytes past 8-byte alignment
            b = i * pitch + 1 + (i + 3 * k + 2) % 7
            src[a:a + chunk].copy_(torch.from_numpy(chunks[i]))
            ins.append(None if i in er else src[a:a + chunk])
            ous.append(dst[b:b + chunk] if i in er and i < c.k else None)
        c.decode_device(ins, er, ous, chunk)
        torch.cuda.synchronize()
        assert clay_amd.last_exec_path() == "stream-local256", (er, clay_amd.last_exec_path())
        ref = np.frombuffer(o.decode({i: chunks[i] for i in range(c.n) if i not in er}, er),
                            dtype=np.uint8).reshape(c.k, -1)
        host = dst.cpu().numpy()
        for i in range(c.n):
            b = i * pitch + 1 + (i + 3 * k + 2) % 7
            if i in er and i < c.k:
                assert np.array_equal(host[b:b + chunk], ref[i]), (sc, er, i)
                assert host[b - 1] == 0x5A and host[b + chunk] == 0x5A, (sc, er, i)

"""GPU parity of the line-local bit-sliced kernels (bitslice_line.hpp) for (4,2,5), BASELINE
config 2, against the oracle: the encode k_bs_encode1 and the single-erasure decode k_bs_decode1.

Inputs are random (not codewords) for the erased data nodes: only the reference's exact RS row
choice (reconstruct from the first k present shards, decode.rs:374) and its iscore order reproduce
those bytes.  Erased parity nodes are checked on codewords against the oracle (the oracle's decode
returns data only) and on random inputs against the grouped plan executor.  Sub-chunks cover whole
2048-position tiles, a partial last tile, byte tails (sc % 8 != 0) and unaligned chunk pointers."""
import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode, last_encode_path, set_encode_path

pytestmark = pytest.mark.gpu

SC = [2048 * 3, 2048 + 8 * 37, 16, 2048 * 2 + 5, 777]


def _run(torch, c, chunks, e, chunk, off=0, mode=None):
    """decode_device of erasure {e}; off > 0 shifts every chunk pointer by off bytes."""
    prev = clay_amd.set_exec_mode(mode) if mode else None
    try:
        base = torch.from_numpy(np.ascontiguousarray(chunks)).cuda()
        if off:
            buf = torch.zeros((c.n, chunk + off), dtype=torch.uint8, device="cuda")
            buf[:, off:] = base
            full = [buf[i, off:] for i in range(c.n)]
            obuf = torch.full((chunk + off,), 0xA5, dtype=torch.uint8, device="cuda")
            out = obuf[off:]
        else:
            full = [base[i] for i in range(c.n)]
            out = torch.full((chunk,), 0xA5, dtype=torch.uint8, device="cuda")
        c.decode_device([None if i == e else full[i] for i in range(c.n)], [e],
                        [out if i == e else None for i in range(c.n)], chunk)
        torch.cuda.synchronize()
        return out.cpu().numpy(), clay_amd.last_exec_path()
    finally:
        if prev is not None:
            clay_amd.set_exec_mode(prev)


@pytest.mark.parametrize("sc", SC)
@pytest.mark.parametrize("off", [0, 3])
def test_decode1_data_nodes_random_inputs(oracle_mod, torch_cuda, sc, off):
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc * 5 + off)
    for e in range(c.k):
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        got, path = _run(torch_cuda, c, chunks, e, chunk, off)
        assert path == "bs-decode1", (e, path)
        ref = np.frombuffer(o.decode({i: chunks[i] for i in range(c.n) if i != e}, [e]), np.uint8).reshape(c.k, -1)
        assert np.array_equal(got, ref[e]), (sc, off, e)


@pytest.mark.parametrize("sc", SC)
def test_decode1_parity_nodes(oracle_mod, torch_cuda, sc):
    """Parity erasures: on a codeword every rebuilt chunk equals the encoded one (oracle encode;
    even sub-chunks); on random inputs the kernel equals the grouped executor."""
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + 11)
    cw = o.encode_array(rng.integers(0, 256, c.k * chunk, dtype=np.uint8))
    # (the oracle pads odd sub-chunks to the next even one: codewords only at even sc)
    for e in range(c.n if cw.shape[1] == chunk else 0):
        got, path = _run(torch_cuda, c, cw, e, chunk)
        assert path == "bs-decode1", (e, path)
        assert np.array_equal(got, cw[e]), (sc, e)
    for e in (c.k, c.k + 1):
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        got, _ = _run(torch_cuda, c, chunks, e, chunk)
        ref, path = _run(torch_cuda, c, chunks, e, chunk, mode="grouped")
        assert path == "grouped"
        assert np.array_equal(got, ref), (sc, e)


def test_decode1_config2_full_size_codeword(oracle_mod, torch_cuda):
    """BASELINE config 2's stripe (64 MiB): every single erasure of a codeword rebuilds the encoded
    chunk (the product encode, itself oracle-checked), and a column slice matches the oracle on
    random inputs."""
    torch = torch_cuda
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    chunk = c.encoded_chunk_size(64 << 20)
    sc = chunk // c.sub_chunk_no
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    full = torch.zeros((c.n, chunk), dtype=torch.uint8, device="cuda")
    full[:c.k] = torch.randint(0, 256, (c.k, chunk), dtype=torch.uint8, device="cuda", generator=g)
    c.encode_device([full[i] for i in range(c.k)], [full[c.k + x] for x in range(c.m)], chunk)
    out = torch.empty(chunk, dtype=torch.uint8, device="cuda")
    for e in range(c.n):
        c.decode_device([None if i == e else full[i] for i in range(c.n)], [e],
                        [out if i == e else None for i in range(c.n)], chunk)
        torch.cuda.synchronize()
        assert clay_amd.last_exec_path() == "bs-decode1"
        assert torch.equal(out, full[e]), e
    # random inputs: positions [p0, p0 + 64) of every sub-chunk are an independent instance
    rnd = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda", generator=g)
    c.decode_device([None if i == 0 else rnd[i] for i in range(c.n)], [0],
                    [out if i == 0 else None for i in range(c.n)], chunk)
    torch.cuda.synchronize()
    host = rnd.view(c.n, c.sub_chunk_no, sc).cpu().numpy()
    got = out.view(c.sub_chunk_no, sc).cpu().numpy()
    for p0 in (0, sc // 2 + 3, sc - 64):
        s = np.ascontiguousarray(host[:, :, p0:p0 + 64]).reshape(c.n, -1)
        ref = np.frombuffer(o.decode({i: s[i] for i in range(1, c.n)}, [0]), np.uint8).reshape(c.k, -1)
        assert np.array_equal(got[:, p0:p0 + 64].reshape(-1), ref[0]), p0


# the oracle pads a sub-chunk to an even length (encode.rs:33-39): even sc for the encode
ENC_SC = [2048 * 3, 2048 + 8 * 37, 16, 2048 * 2 + 6, 778]


@pytest.mark.parametrize("sc", ENC_SC)
def test_encode1_matches_oracle(oracle_mod, sc):
    """Auto mode runs k_bs_encode1 for (4,2,5): whole tiles, a partial last tile, byte tails
    (sc % 8 != 0), bit-exact against the oracle; "bitsliced" still selects the v1 kernel."""
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    data = np.random.default_rng(sc).integers(0, 256, c.k * c.sub_chunk_no * sc, dtype=np.uint8).tobytes()
    ref = o.encode_array(data)
    assert ref.shape[1] == c.sub_chunk_no * sc
    got = c.encode_array(data)
    assert last_encode_path().startswith("bitsliced-line"), last_encode_path()
    assert np.array_equal(got, ref), sc
    set_encode_path("bitsliced", 0)
    try:
        v1 = c.encode_array(data)
        assert last_encode_path().startswith("bitsliced-k4m2"), last_encode_path()
    finally:
        set_encode_path("auto", 0)
    assert np.array_equal(v1, ref)


@pytest.mark.parametrize("off", [1, 6])
def test_encode1_unaligned_chunks(oracle_mod, torch_cuda, off):
    """Chunk pointers off 8-byte alignment take the byte-tail instantiation."""
    torch = torch_cuda
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    sc = 2048 + 40
    chunk = c.sub_chunk_no * sc
    data = np.random.default_rng(off).integers(0, 256, c.k * chunk, dtype=np.uint8)
    ref = o.encode_array(data.tobytes())
    buf = torch.zeros((c.n, chunk + off), dtype=torch.uint8, device="cuda")
    buf[:c.k, off:] = torch.from_numpy(data.reshape(c.k, chunk)).cuda()
    c.encode_device([buf[i, off:] for i in range(c.k)], [buf[c.k + x, off:] for x in range(c.m)], chunk)
    torch.cuda.synchronize()
    assert last_encode_path().startswith("bitsliced-line"), last_encode_path()
    assert np.array_equal(buf[c.k:, off:].cpu().numpy(), ref[c.k:])


def test_encode1_config2_full_size_slices(oracle_mod, torch_cuda):
    """BASELINE config 2's 64 MiB stripe: column slices of the parity match the oracle's encode of
    the same slices (positions [p0, p0 + 64) of every sub-chunk are an independent codeword)."""
    torch = torch_cuda
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    chunk = c.encoded_chunk_size(64 << 20)
    sc = chunk // c.sub_chunk_no
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    full = torch.zeros((c.n, chunk), dtype=torch.uint8, device="cuda")
    full[:c.k] = torch.randint(0, 256, (c.k, chunk), dtype=torch.uint8, device="cuda", generator=g)
    c.encode_device([full[i] for i in range(c.k)], [full[c.k + x] for x in range(c.m)], chunk)
    torch.cuda.synchronize()
    assert last_encode_path().startswith("bitsliced-line"), last_encode_path()
    host = full.view(c.n, c.sub_chunk_no, sc).cpu().numpy()
    for p0 in (0, sc // 2 + 8, sc - 64):
        s = np.ascontiguousarray(host[:, :, p0:p0 + 64]).reshape(c.n, -1)
        ref = o.encode_array(s[:c.k].reshape(-1).tobytes())
        assert np.array_equal(s[c.k:], ref[c.k:]), p0

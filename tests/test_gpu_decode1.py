"""GPU parity of the single-erasure bit-sliced decode k_bs_decode1 (bitslice_decode1.hpp) for
(4,2,5), BASELINE config 2, against the oracle.

Inputs are random (not codewords) for the erased data nodes: only the reference's exact RS row
choice (reconstruct from the first k present shards, decode.rs:374) and its iscore order reproduce
those bytes.  Erased parity nodes are checked on codewords against the oracle (the oracle's decode
returns data only) and on random inputs against the grouped plan executor.  Sub-chunks cover whole
2048-position tiles, a partial last tile, byte tails (sc % 8 != 0) and unaligned chunk pointers."""
import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode

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

"""GPU tests of clay_decode_device_codeword (ClayCode.decode_device(..., codeword=True)): a decode of
one erased node with every other chunk present, in a q = m code, is rebuilt by the streaming repair
kernel (k_bs_repair_stream) from the whole chunks.  The reference's decode (decode.rs:31-161) and
repair (repair.rs:140-421) return the same bytes whenever the chunks are one codeword, so the inputs
here are codewords encoded by the oracle and every rebuilt chunk (data or parity) must equal the
encoded one bit for bit.  Other patterns and sizes run as clay_decode_device.  The choice is per
call: a concurrent clay_decode_device of arbitrary chunks keeps the reference decode's bytes."""
import threading

import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode

pytestmark = pytest.mark.gpu


def _decode_dev(torch, c, full, er, chunk, codeword=True, stream=None):
    """Output buffer fill, decode and read-back all on one stream (the thread's own in the
    concurrency test), so nothing races with the fill."""
    st = stream if stream is not None else torch.cuda.current_stream()
    with torch.cuda.stream(st):
        outs = torch.full((c.n, chunk), 0xA5, dtype=torch.uint8, device="cuda")
        c.decode_device([None if i in er else full[i] for i in range(c.n)], er,
                        [outs[i] if i in er else None for i in range(c.n)], chunk, 0, st.cuda_stream,
                        codeword=codeword)
        host = outs.cpu()
    st.synchronize()
    return host


# sub-chunks that give every CU of a 256-CU MI355X at least one tile of the streaming repair
# kernel (256 B for (10,4,13), 512 B for (9,3,11)), ragged ends included (sc = 2 mod 8 for (9,3,11))
@pytest.mark.parametrize("cfg,sc,lost", [((10, 4, 13), 65536 + 40, [0, 5, 9, 10, 13]),
                                         ((9, 3, 11), 131072 + 2, [0, 4, 8, 11])])
def test_codeword_single_erasure_runs_repair(oracle_mod, torch_cuda, cfg, sc, lost):
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(sc).integers(0, 256, c.k * chunk, dtype=np.uint8))
    full = torch.from_numpy(ref).cuda()
    for e in lost:
        outs = _decode_dev(torch, c, full, [e], chunk)
        assert clay_amd.last_exec_path() == "bs-repair-stream", (e, clay_amd.last_exec_path())
        assert np.array_equal(outs[e].numpy(), ref[e]), (cfg, e)
        # the other outputs were not requested and stay untouched
        assert int((outs[(e + 1) % c.n] != 0xA5).sum().item()) == 0


@pytest.mark.parametrize("mode", ["grouped", "tile"])
def test_codeword_route_follows_exec_mode(oracle_mod, torch_cuda, mode):
    """Under exec modes that do not pick the bit-sliced repair kernels ("grouped", "tile": A/B
    runs) the codeword entry point runs as clay_decode_device, like clay_repair_device's kernel
    choice; the bytes are the codeword's either way."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    sc = 65536 + 40
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(5).integers(0, 256, c.k * chunk, dtype=np.uint8))
    full = torch.from_numpy(ref).cuda()
    prev = clay_amd.set_exec_mode(mode)
    try:
        outs = _decode_dev(torch, c, full, [3], chunk)
        assert clay_amd.last_exec_path() != "bs-repair-stream", (mode, clay_amd.last_exec_path())
    finally:
        clay_amd.set_exec_mode(prev)
    assert np.array_equal(outs[3].numpy(), ref[3])


def test_codeword_other_patterns_as_auto(oracle_mod, torch_cuda):
    """Two erasures, and one erasure at a sub-chunk too small for every CU to get a tile: the
    paths auto takes (local decode), bit-exact."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    for sc, er in ((65536 + 40, [0, 4]), (64 * 40 + 8, [3])):
        chunk = c.sub_chunk_no * sc
        ref = o.encode_array(np.random.default_rng(sc + len(er)).integers(0, 256, c.k * chunk, dtype=np.uint8))
        full = torch.from_numpy(ref).cuda()
        outs = _decode_dev(torch, c, full, er, chunk)
        assert clay_amd.last_exec_path() == "stream-local256", (sc, er, clay_amd.last_exec_path())
        for e in er:
            assert np.array_equal(outs[e].numpy(), ref[e]), (sc, er, e)


def test_plain_decode_keeps_decode_semantics_on_non_codewords(oracle_mod, torch_cuda):
    """clay_decode_device never takes the repair route: on random (non-codeword) chunks a
    single-erasure decode at the same size still returns the reference decode's bytes."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    sc = 65536 + 40
    chunk = c.sub_chunk_no * sc
    chunks = np.random.default_rng(3).integers(0, 256, (c.n, chunk), dtype=np.uint8)
    outs = _decode_dev(torch, c, torch.from_numpy(chunks).cuda(), [2], chunk, codeword=False)
    assert clay_amd.last_exec_path() == "stream-local256"
    av = {i: chunks[i] for i in range(c.n) if i != 2}
    ref = np.frombuffer(o.decode(av, [2]), dtype=np.uint8).reshape(c.k, -1)
    assert np.array_equal(outs[2].numpy(), ref[2])


def test_codeword_call_does_not_change_concurrent_decodes(oracle_mod, torch_cuda):
    """Thread A decodes a codeword through the codeword entry point while thread B decodes random
    (non-codeword) chunks through clay_decode_device, interleaved, each on its own stream: B's
    bytes are the reference decode's every time (with a process-wide mode they were not)."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    sc = 65536 + 40
    chunk = c.sub_chunk_no * sc
    ref = o.encode_array(np.random.default_rng(11).integers(0, 256, c.k * chunk, dtype=np.uint8))
    cw = torch.from_numpy(ref).cuda()
    rnd = np.random.default_rng(12).integers(0, 256, (c.n, chunk), dtype=np.uint8)
    rd = torch.from_numpy(rnd).cuda()
    want_b = np.frombuffer(o.decode({i: rnd[i] for i in range(c.n) if i != 2}, [2]), dtype=np.uint8).reshape(c.k, -1)[2]
    errors, paths = [], {"a": set(), "b": set()}
    start = threading.Barrier(2)

    def thread_a():
        s = torch.cuda.Stream()
        start.wait()
        for _ in range(12):
            out = _decode_dev(torch, c, cw, [2], chunk, codeword=True, stream=s)
            paths["a"].add(clay_amd.last_exec_path())
            if not np.array_equal(out[2].numpy(), ref[2]):
                errors.append("codeword decode")

    def thread_b():
        s = torch.cuda.Stream()
        start.wait()
        for _ in range(12):
            out = _decode_dev(torch, c, rd, [2], chunk, codeword=False, stream=s)
            paths["b"].add(clay_amd.last_exec_path())
            if not np.array_equal(out[2].numpy(), want_b):
                errors.append("plain decode of random chunks changed")

    ts = [threading.Thread(target=thread_a), threading.Thread(target=thread_b)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    assert paths == {"a": {"bs-repair-stream"}, "b": {"stream-local256"}}, paths

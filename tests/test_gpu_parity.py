"""GPU parity: the HIP path (through the C ABI) against the oracle, bit-exact.

Small/medium sizes compare whole outputs with the oracle on the same seeded
inputs; the BASELINE.json configurations run at full size (marked slow as well).
Non-codeword (random) decode/repair inputs pin the reference's RS row selection.
"""
import itertools

import numpy as np
import pytest

from clay_amd import ClayCode, set_encode_path, last_encode_path
import clay_amd

pytestmark = pytest.mark.gpu

CONFIGS = [(4, 2, 5), (6, 3, 8), (9, 3, 11), (10, 4, 13), (5, 3, 6), (7, 4, 9), (3, 3, 4), (8, 4, 11)]


def rand_bytes(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def internal(c, e):
    return e if e < c.k else e + c.nu


@pytest.fixture(autouse=True)
def _auto_path():
    set_encode_path("auto")
    yield
    set_encode_path("auto")


@pytest.fixture(params=["tile", "grouped"])
def exec_mode(request):
    """Run a decode/repair test under both plan executors (tile-fused and grouped)."""
    prev = clay_amd.set_exec_mode(request.param)
    yield request.param
    clay_amd.set_exec_mode(prev)


@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("size_kind", ["empty", "tiny", "ragged", "aligned16", "sc2", "big"])
def test_encode_matches_oracle(oracle_mod, cfg, size_kind):
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    unit = k * c.sub_chunk_no * 2
    n = {"empty": 0, "tiny": 1, "ragged": unit * 3 + 17, "aligned16": unit * 8,
         "sc2": unit * 5, "big": unit * 40 - 3}[size_kind]
    data = rand_bytes(hash(cfg) & 0xFFFF, n)
    ref = o.encode_array(data)
    got = c.encode_array(data)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), (cfg, size_kind, clay_amd.last_encode_path())


BS_CODES = [(10, 4, 13), (4, 2, 5), (8, 4, 11), (9, 3, 11), (6, 3, 8)]


@pytest.mark.parametrize("cfg", BS_CODES)
@pytest.mark.parametrize("tile", [0, 1, 4])
@pytest.mark.parametrize("scale", [1, 3, 37])
def test_bitsliced_encode_matches_oracle(oracle_mod, cfg, tile, scale):
    """Bit-sliced kernel: full tiles, the ragged last tile, every tile width."""
    if tile and cfg != (10, 4, 13):
        pytest.skip("tile override only instantiated for (10,4,13)")
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    n = k * c.sub_chunk_no * 8 * scale * 4 - 11  # sc = 32*scale: several tiles + a partial one
    data = rand_bytes(scale * 7 + tile, n)
    ref = o.encode_array(data)
    set_encode_path("bitsliced", tile)
    got = c.encode_array(data)
    assert last_encode_path().startswith("bitsliced"), last_encode_path()
    assert np.array_equal(got, ref), (cfg, tile, scale)


# even: the reference pads to k * alpha * 2 (encode.rs:33-39); 2 mod 8 like the BASELINE chunk
STREAM3_SC = [16, 18, 100, 510, 512, 514, 1000, 4098, 512 * 256 + 38, 512 * 300 * 8 + 2, 51_782]


@pytest.mark.parametrize("loaders", [2, 7])
@pytest.mark.parametrize("sc", STREAM3_SC)
def test_stream3_encode_matches_oracle(oracle_mod, loaders, sc):
    """(9,3,11) streaming kernel (stream_encode3.hpp): sub-chunk sizes from 16 (one partial tile,
    2 mod 8 rows like the 256 MiB BASELINE chunk, more tiles than workgroups),
    2 / 7 loader waves, bit-exact against the oracle."""
    c, o = ClayCode(9, 3, 11), oracle_mod.OracleClay(9, 3, 11)
    n = 9 * c.sub_chunk_no * sc - 5
    data = rand_bytes(sc * 3 + loaders, n)
    ref = o.encode_array(data)
    assert ref.shape[1] == c.sub_chunk_no * sc
    set_encode_path("stream", loaders)
    try:
        got = c.encode_array(data)
        assert last_encode_path().startswith("stream3"), last_encode_path()
    finally:
        set_encode_path("auto", 0)
    assert np.array_equal(got, ref), (sc, loaders)


@pytest.mark.parametrize("loaders", [2, 7])
@pytest.mark.parametrize("sc", [17, 511, 513, 512 * 256 + 37])
def test_stream3_encode_odd_subchunk(oracle_mod, torch_cuda, loaders, sc):
    """Odd sub-chunks, which only the device API reaches (ClayCode::encode pads to an even sc,
    encode.rs:33-39), on the (9,3,11) streaming kernel.  Every byte offset of the sub-chunks is an
    independent codeword, so the reference parity of the odd layout is the oracle's parity of the
    even layout sc + 1 restricted to positions [0, sc) of every sub-chunk (encode.rs:57-68)."""
    torch = torch_cuda
    c, o = ClayCode(9, 3, 11), oracle_mod.OracleClay(9, 3, 11)
    alpha = c.sub_chunk_no
    wide = o.encode_array(rand_bytes(sc + 5 * loaders, 9 * alpha * (sc + 1)))
    assert wide.shape[1] == alpha * (sc + 1)
    narrow = np.ascontiguousarray(wide.reshape(c.n, alpha, sc + 1)[:, :, :sc].reshape(c.n, alpha * sc))
    chunk = alpha * sc
    dev = torch.from_numpy(narrow[:9].copy()).cuda()
    par = torch.full((3, chunk), 0xA5, dtype=torch.uint8, device="cuda")
    set_encode_path("stream", loaders)
    try:
        c.encode_device([dev[i] for i in range(9)], [par[i] for i in range(3)], chunk)
        torch.cuda.synchronize()
        assert last_encode_path().startswith("stream3"), last_encode_path()
    finally:
        set_encode_path("auto", 0)
    assert np.array_equal(par.cpu().numpy(), narrow[9:]), (sc, loaders)


STREAM_SC = [16, 24, 64, 72, 104, 128, 256, 1064, 6440, 8 * 256 * 32, 8 * 256 * 32 + 8, 64 * 300 + 40,
             64 * 2000 + 8, 8 * 256 * 32 * 3 + 4096 + 24]


@pytest.mark.parametrize("cfg", [(10, 4, 13), (9, 4, 12)])
@pytest.mark.parametrize("loaders", [0, 1, 2])
@pytest.mark.parametrize("sc", STREAM_SC)
def test_stream_encode_matches_oracle(oracle_mod, cfg, loaders, sc):
    """Streaming kernel (q = 4, t = 4): tiny sub-chunks (one partial tile), exact XCD
    rounds, sc % 16 == 8 (straddling piece patched in LDS), partial tiles of every
    width and more tiles than workgroups; 1 / 2 / 4 loader waves."""
    k, m, d = cfg
    if loaders and cfg != (10, 4, 13):
        pytest.skip("loader variants are instantiated for (10,4,13)")
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    n = k * c.sub_chunk_no * sc - 7
    data = rand_bytes(sc + loaders, n)
    ref = o.encode_array(data)
    assert ref.shape[1] == c.sub_chunk_no * sc
    set_encode_path("stream", loaders)
    got = c.encode_array(data)
    assert last_encode_path().startswith("stream"), last_encode_path()
    assert np.array_equal(got, ref), (cfg, sc, loaders)


def test_encode_path_rejects_unknown_variants():
    """Only paths that produce the reference's parity are selectable."""
    with pytest.raises(ValueError):
        set_encode_path("bitsliced", 40)
    with pytest.raises(ValueError):
        set_encode_path("stream", 3)
    with pytest.raises(ValueError):
        set_encode_path("probe")
    assert clay_amd._lib.lib().clay_set_encode_path(9 | 2 << 8) == -1
    assert clay_amd._lib.lib().clay_set_encode_path(12) == -1


@pytest.mark.parametrize("cfg", CONFIGS)
def test_encode_fused_equals_staged(oracle_mod, cfg, exec_mode):
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    data = rand_bytes(7, k * c.sub_chunk_no * 2 * 16 - 5)  # sc = 32: fused-eligible
    ref = o.encode_array(data)
    set_encode_path("staged")
    a = c.encode_array(data)
    assert last_encode_path() == "staged"
    set_encode_path("fused" if (c.q == c.m and c.q <= 4) else "auto")
    b = c.encode_array(data)
    assert np.array_equal(a, ref) and np.array_equal(b, ref), last_encode_path()
    if c.q == c.m and c.q <= 4:
        assert last_encode_path().startswith("fused"), last_encode_path()
    set_encode_path("auto")
    assert np.array_equal(c.encode_array(data), ref), last_encode_path()


@pytest.mark.parametrize("cfg", CONFIGS)
def test_decode_random_inputs_match_oracle(oracle_mod, cfg, exec_mode):
    """Non-codeword inputs: only the reference's exact RS row choice reproduces these bytes."""
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    rng = np.random.default_rng(11)
    chunk = c.sub_chunk_no * 6
    pats = [list(e) for r in range(0, m + 1) for e in itertools.combinations(range(c.n), r)]
    rng.shuffle(pats)
    for er in pats[:12]:
        chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
        av = {i: chunks[i] for i in range(c.n) if i not in er}
        assert c.decode(av, er) == o.decode(av, er), (cfg, er)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_decode_roundtrip_max_erasures(oracle_mod, cfg, exec_mode):
    k, m, d = cfg
    c = ClayCode(k, m, d)
    data = rand_bytes(3, k * c.sub_chunk_no * 4 + 9)
    chunks = c.encode(data)
    for er in list(itertools.combinations(range(c.n), m))[:20]:
        av = {i: chunks[i] for i in range(c.n) if i not in er}
        assert c.decode(av, list(er))[:len(data)] == data.tobytes(), (cfg, er)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_repair_every_node_matches_oracle(oracle_mod, cfg, exec_mode):
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    data = rand_bytes(5, k * c.sub_chunk_no * 2 * 3)
    chunks = c.encode_array(data)
    chunk = chunks.shape[1]
    sc = chunk // c.sub_chunk_no
    rng = np.random.default_rng(9)
    for lost in range(c.n):
        avail = [i for i in range(c.n) if i != lost]
        info = c.minimum_to_repair(lost, avail)
        assert info == o.minimum_to_repair(lost, avail)
        pd = {h: np.concatenate([chunks[h][z * sc:(z + 1) * sc] for z in idx]) for h, idx in info}
        rec = c.repair(lost, pd, chunk)
        assert rec == chunks[lost].tobytes(), (cfg, lost)
        # random helper payloads: byte-identical to the reference's repair arithmetic
        pr = {h: rng.integers(0, 256, v.size, dtype=np.uint8) for h, v in pd.items()}
        assert c.repair(lost, pr, chunk) == o.repair(lost, pr, chunk), (cfg, lost)


@pytest.mark.parametrize("cfg,lost,mode,launches", [((9, 3, 11), 0, "tile", 1), ((4, 2, 5), 3, "auto", 1),
                                                     ((10, 4, 13), 0, "tile", 1), ((9, 3, 11), 0, "auto", 1)])
def test_tile_executor_selected(oracle_mod, cfg, lost, mode, launches):
    """'tile' runs repair plans whose U slots fit in LDS as ONE tile-fused launch; 'auto' runs
    the bit-sliced repair kernel (one launch) for the q = m codes it is instantiated for; the
    bytes equal the grouped executor's and the oracle's."""
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    sc = 16 * 100 + 6
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(77)
    avail = [i for i in range(c.n) if i != lost]
    info = c.minimum_to_repair(lost, avail)
    pr = {h: rng.integers(0, 256, len(idx) * sc, dtype=np.uint8) for h, idx in info}
    prev = clay_amd.set_exec_mode(mode)
    try:
        got = c.repair(lost, pr, chunk)
        assert clay_amd.last_launch_count() == launches
        assert clay_amd.last_exec_path() == ("tile" if mode == "tile" else "bs-repair")
        clay_amd.set_exec_mode("grouped")
        assert c.repair(lost, pr, chunk) == got
    finally:
        clay_amd.set_exec_mode(prev)
    assert got == o.repair(lost, pr, chunk)


@pytest.mark.parametrize("mode,expect", [("auto", "bs-decode1"), ("grouped", "grouped"), ("tile", "tile")])
def test_small_decode_plan_executor(oracle_mod, mode, expect):
    """(4,2,5) 1-erasure decode: auto runs the bit-sliced single-erasure kernel (round 6), "tile"
    the small two-level plan on the tile-fused executor (one launch); every mode returns the
    oracle's bytes on random inputs."""
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    chunk = c.sub_chunk_no * (16 * 300 + 6)
    chunks = np.random.default_rng(5).integers(0, 256, (c.n, chunk), dtype=np.uint8)
    av = {i: chunks[i] for i in range(c.n) if i != 0}
    prev = clay_amd.set_exec_mode(mode)
    try:
        got = c.decode(av, [0])
        assert clay_amd.last_exec_path() == expect
    finally:
        clay_amd.set_exec_mode(prev)
    assert got == o.decode(av, [0])


def test_exec_mode_rejects_unknown():
    with pytest.raises(ValueError):
        clay_amd.set_exec_mode("fused")
    assert clay_amd._lib.lib().clay_set_exec_mode(8) == -1


def test_repair_with_all_helpers_and_aloof(oracle_mod):
    """More than d helpers, and exactly d with an aloof node (repair.rs:248-255)."""
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    data = rand_bytes(21, 10 * 256 * 2 * 2)
    ch = c.encode_array(data)
    chunk = ch.shape[1]
    sc = chunk // 256
    for lost in (0, 5, 9, 10, 13):
        idx = c.minimum_to_repair(lost, [i for i in range(14) if i != lost])[0][1]
        for helpers in ([i for i in range(14) if i != lost],
                        [h for h, _ in c.minimum_to_repair(lost, [i for i in range(14) if i != lost])]):
            pd = {h: np.concatenate([ch[h][z * sc:(z + 1) * sc] for z in idx]) for h in helpers}
            got = c.repair(lost, pd, chunk)
            assert got == o.repair(lost, pd, chunk) == ch[lost].tobytes()


def test_errors_mirror_reference(oracle_mod):
    c = ClayCode(4, 2, 5)
    ch = c.encode(bytes(range(128)))
    with pytest.raises(clay_amd.TooManyErasures) as e:
        c.decode({i: ch[i] for i in range(3, 6)}, [0, 1, 2])
    assert e.value.fields[:2] == (2, 3)
    bad = {i: ch[i] for i in range(1, 6)}
    bad[5] = ch[5] + b"\0"
    with pytest.raises((clay_amd.InconsistentChunkSizes, clay_amd.InvalidChunkSize)):
        c.decode(bad, [0])
    with pytest.raises(clay_amd.InvalidParameters, match="both"):
        c.decode({i: ch[i] for i in range(6)}, [0])
    with pytest.raises(clay_amd.InvalidParameters, match="Expected"):
        c.decode({i: ch[i] for i in range(2, 6)}, [0])


# ---------------------------------------------------------------------------
# device-resident API (torch allocations; pointers through the C ABI)
# ---------------------------------------------------------------------------
def test_device_api_encode_decode_repair(oracle_mod, torch_cuda):
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    data = rand_bytes(31, 10 * 256 * 2 * 40)
    ref = o.encode_array(data)
    chunk = ref.shape[1]
    dev = torch.from_numpy(ref[:10].copy()).cuda()
    par = torch.zeros((4, chunk), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    c.encode_device([dev[i] for i in range(10)], [par[i] for i in range(4)], chunk, 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy(), ref[10:])
    # batched
    dev2 = torch.stack([dev, dev.flip(1)])
    par2 = torch.zeros((2, 4, chunk), dtype=torch.uint8, device="cuda")
    c.encode_device_batch([dev2[s, i] for s in range(2) for i in range(10)],
                          [par2[s, i] for s in range(2) for i in range(4)], 2, chunk, 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(par2[0].cpu().numpy(), ref[10:])
    ref_flip = o.encode_array(np.ascontiguousarray(ref[:10, ::-1]).reshape(-1))
    assert np.array_equal(par2[1].cpu().numpy(), ref_flip[10:])
    # decode on device: erase {0,4,8,12}, rebuild data and parity 12
    full = torch.from_numpy(ref.copy()).cuda()
    er = [0, 4, 8, 12]
    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(14)], er,
                    [outs[i] if i in er else None for i in range(14)], chunk, 0, stream)
    torch.cuda.synchronize()
    for e in er:
        assert np.array_equal(outs[e].cpu().numpy(), ref[e]), e
    # repair on device
    sc = chunk // 256
    info = c.minimum_to_repair(3, [i for i in range(14) if i != 3])
    hb = [torch.from_numpy(np.concatenate([ref[h][z * sc:(z + 1) * sc] for z in idx])).cuda()
          for h, idx in info]
    out = torch.zeros(chunk, dtype=torch.uint8, device="cuda")
    c.repair_device(3, [h for h, _ in info], hb, chunk, out, 0, stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref[3])


# ---------------------------------------------------------------------------
# BASELINE.json configurations at full size
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("size", [1024, 10 * 1024, 100 * 1024, 1 << 20])
def test_cfg1_4_2_5_clay_bench_sizes(oracle_mod, torch_cuda, size):
    """BASELINE configs[0] / benches/clay_bench.rs:20-56 shape: (4,2,5) encode of 1 KiB -
    1 MiB (1 MiB: chunk 262,144, sub-chunk 32,768) through every entry point -- host
    clay_encode, clay_encode_device (one stripe), clay_encode_device_batch and
    clay_encode_device_strided (64 stripes) -- plus the bench's decode (1 erasure) and
    repair legs, all against the oracle."""
    torch = torch_cuda
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    data = rand_bytes(size, size)
    ref = o.encode_array(data)
    chunk = ref.shape[1]
    if size == 1 << 20:
        assert chunk == 262_144 and chunk // c.sub_chunk_no == 32_768
    assert np.array_equal(c.encode_array(data), ref)
    dev = torch.from_numpy(ref[:4].copy()).cuda()
    par = torch.zeros((2, chunk), dtype=torch.uint8, device="cuda")
    c.encode_device([dev[i] for i in range(4)], [par[i] for i in range(2)], chunk)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy(), ref[4:])
    n = 64
    refs = [o.encode_array(rand_bytes(size + s, size)) for s in range(n)]
    bd = torch.from_numpy(np.stack([r[:4] for r in refs])).cuda()
    bp = torch.zeros((n, 2, chunk), dtype=torch.uint8, device="cuda")
    c.encode_device_batch([bd[s, i] for s in range(n) for i in range(4)], [bp[s, j] for s in range(n) for j in range(2)],
                          n, chunk)
    torch.cuda.synchronize()
    assert np.array_equal(bp.cpu().numpy(), np.stack([r[4:] for r in refs]))
    bp.zero_()
    c.encode_device_strided(bd, bp, n, chunk)
    torch.cuda.synchronize()
    assert np.array_equal(bp.cpu().numpy(), np.stack([r[4:] for r in refs]))
    av = {i: ref[i] for i in range(1, 6)}                       # clay_bench.rs decode leg
    assert c.decode(av, [0]) == o.decode(av, [0])
    info = c.minimum_to_repair(0, [1, 2, 3, 4, 5])              # clay_bench.rs repair leg
    sc = chunk // c.sub_chunk_no
    pd = {h: np.concatenate([ref[h][z * sc:(z + 1) * sc] for z in idx]) for h, idx in info}
    assert c.repair(0, pd, chunk) == o.repair(0, pd, chunk) == ref[0].tobytes()


@pytest.mark.slow
def test_cfg2_4_2_5_64MiB_encode_decode(oracle_mod):
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    data = rand_bytes(42, 64 << 20)
    ref = o.encode_array(data)
    got = c.encode_array(data)
    assert np.array_equal(got, ref), clay_amd.last_encode_path()
    av = {i: ref[i] for i in range(1, 6)}
    assert c.decode(av, [0]) == o.decode(av, [0])


@pytest.mark.slow
def test_cfg4_10_4_13_1GiB_encode_device(oracle_mod, torch_cuda):
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    data = rand_bytes(42, 1 << 30)
    chunk = c.encoded_chunk_size(data.size)
    assert chunk == 107_374_592
    ref = o.encode_array(data)
    dev = torch.from_numpy(ref[:10].copy()).cuda()
    # every encode kernel at the BASELINE size (sc = 419,432: ragged last tile, 8-byte
    # aligned sub-chunks), auto first
    for path, tile, prefix in [("auto", 0, "stream-k10m4-w256-l4"), ("stream", 1, "stream-k10m4-w256-l1"),
                               ("stream", 2, "stream-k10m4-w256-l2"), ("bitsliced", 0, "bitsliced-k10m4"),
                               ("fused", 0, "fused")]:
        par = torch.zeros((4, chunk), dtype=torch.uint8, device="cuda")
        set_encode_path(path, tile)
        c.encode_device([dev[i] for i in range(10)], [par[i] for i in range(4)], chunk)
        torch.cuda.synchronize()
        assert clay_amd.last_encode_path().startswith(prefix), (path, clay_amd.last_encode_path())
        assert np.array_equal(par.cpu().numpy(), ref[10:]), path


@pytest.mark.slow
@pytest.mark.parametrize("mode,path", [("auto", "stream-fused2"), ("grouped", "grouped")])
def test_cfg5_10_4_13_1GiB_decode_4_erasures(oracle_mod, torch_cuda, mode, path):
    """BASELINE config 5 on random (non-codeword) chunks under the auto executor (the fused
    decode v2) and the grouped plan executor."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    rng = np.random.default_rng(5)
    chunk = 107_374_592
    er = [0, 4, 8, 12]
    # non-codeword inputs: pins row selection at full size too
    chunks = rng.integers(0, 256, (14, chunk), dtype=np.uint8)
    av = {i: chunks[i] for i in range(14) if i not in er}
    ref = np.frombuffer(o.decode(av, er), np.uint8).reshape(10, chunk)
    full = torch.from_numpy(chunks).cuda()
    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
    prev = clay_amd.set_exec_mode(mode)
    try:
        c.decode_device([None if i in er else full[i] for i in range(14)], er,
                        [outs[i] if i in er else None for i in range(14)], chunk)
        torch.cuda.synchronize()
        assert clay_amd.last_exec_path() == path
    finally:
        clay_amd.set_exec_mode(prev)
    for e in (0, 4, 8):
        assert np.array_equal(outs[e].cpu().numpy(), ref[e]), e


@pytest.mark.slow
def test_cfg5_10_4_13_1GiB_decode_4_erasures_codeword_incl_parity(oracle_mod, torch_cuda):
    """The same 4-erasure pattern on a real 1 GiB codeword (encoded by the oracle): every
    erased node comes back, the rebuilt parity node 12 (internal 14) included."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    data = rand_bytes(55, 1 << 30)
    ref = o.encode_array(data)
    chunk = ref.shape[1]
    er = [0, 4, 8, 12]
    full = torch.from_numpy(ref).cuda()
    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(14)], er,
                    [outs[i] if i in er else None for i in range(14)], chunk)
    torch.cuda.synchronize()
    assert clay_amd.last_exec_path() == "stream-fused2"  # auto, one erasure in every section
    for e in er:
        assert np.array_equal(outs[e].cpu().numpy(), ref[e]), e


@pytest.mark.slow
@pytest.mark.parametrize("er", [[0], [0, 4], [0, 1]])
def test_local256_10_4_13_1GiB_decode(oracle_mod, torch_cuda, er):
    """The local decode on 256-byte row runs at the BASELINE stripe (sc 419,432: partial tiles
    ending at sc % 16 == 8) on random (non-codeword) chunks: every erased data chunk equals the
    oracle's decode."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    chunk = 107_374_592
    chunks = np.random.default_rng(17 + len(er)).integers(0, 256, (14, chunk), dtype=np.uint8)
    av = {i: chunks[i] for i in range(14) if i not in er}
    ref = np.frombuffer(o.decode(av, er), np.uint8).reshape(10, chunk)
    full = torch.from_numpy(chunks).cuda()
    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(14)], er,
                    [outs[i] if i in er else None for i in range(14)], chunk)
    torch.cuda.synchronize()
    assert clay_amd.last_exec_path() == "stream-local256"
    for e in er:
        assert np.array_equal(outs[e].cpu().numpy(), ref[e]), e


@pytest.mark.slow
def test_local256_10_4_13_1GiB_codeword_parity_pair(oracle_mod, torch_cuda):
    """Two parity nodes of one section ({12, 13}: internal 14, 15, a both-erased pair) on a real
    1 GiB codeword: both rebuilt parity chunks equal the encoded ones."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    ref = o.encode_array(rand_bytes(57, 1 << 30))
    chunk = ref.shape[1]
    er = [12, 13]
    full = torch.from_numpy(ref).cuda()
    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
    c.decode_device([None if i in er else full[i] for i in range(14)], er,
                    [outs[i] if i in er else None for i in range(14)], chunk)
    torch.cuda.synchronize()
    assert clay_amd.last_exec_path() == "stream-local256"
    for e in er:
        assert np.array_equal(outs[e].cpu().numpy(), ref[e]), e


@pytest.mark.slow
def test_cfg3_9_3_11_encode_full_size(oracle_mod, torch_cuda):
    """(9,3,11) stripe of 9 x 256 MiB: chunk 268,435,458, sc 3,314,018 (= 2 mod 8, off the
    bit-sliced kernels' 8-byte gate), whole parity against the oracle."""
    torch = torch_cuda
    c, o = ClayCode(9, 3, 11), oracle_mod.OracleClay(9, 3, 11)
    data = rand_bytes(93, 9 * (256 << 20))
    ref = o.encode_array(data)
    chunk = ref.shape[1]
    assert chunk == 268_435_458
    dev = torch.from_numpy(ref[:9].copy()).cuda()
    par = torch.zeros((3, chunk), dtype=torch.uint8, device="cuda")
    c.encode_device([dev[i] for i in range(9)], [par[i] for i in range(3)], chunk)
    torch.cuda.synchronize()
    assert np.array_equal(par.cpu().numpy(), ref[9:]), clay_amd.last_encode_path()


@pytest.mark.slow
@pytest.mark.parametrize("lost", [0, 11])
def test_cfg3_9_3_11_repair_256MiB_chunks(oracle_mod, torch_cuda, lost):
    """Node 0 (data) and node 11 (last parity, the slowest plan in bench_paths)."""
    torch = torch_cuda
    c, o = ClayCode(9, 3, 11), oracle_mod.OracleClay(9, 3, 11)
    chunk = 268_435_458
    sc = chunk // 81
    rng = np.random.default_rng(8 + lost)
    info = c.minimum_to_repair(lost, [i for i in range(12) if i != lost])
    assert len(info) == 11 and len(info[0][1]) == 27
    pd = {h: rng.integers(0, 256, 27 * sc, dtype=np.uint8) for h, _ in info}
    ref = np.frombuffer(o.repair(lost, pd, chunk), np.uint8)
    hb = [torch.from_numpy(pd[h]).cuda() for h, _ in info]
    out = torch.zeros(chunk, dtype=torch.uint8, device="cuda")
    c.repair_device(lost, [h for h, _ in info], hb, chunk, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("cfg", [(4, 2, 5), (9, 3, 11), (10, 4, 13)])
@pytest.mark.parametrize("sc", [16 * 257 + 2, 16 * 1000 + 9, 16 * 3001])
def test_decode_repair_multi_tile_unaligned_subchunks(oracle_mod, cfg, sc, exec_mode):
    """Sub-chunks spanning several executor tiles whose regions start at 2-byte / odd
    offsets (the (9,3,11) 256 MiB chunk has sc = 3,314,018): random (non-codeword)
    inputs, decode and repair byte-identical to the oracle."""
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc)
    chunks = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)
    er = list(range(0, c.n, c.q))[:m]
    av = {i: chunks[i] for i in range(c.n) if i not in er}
    assert c.decode(av, er) == o.decode(av, er), (cfg, sc, er)
    for lost in (0, c.n - 1):
        avail = [i for i in range(c.n) if i != lost]
        info = c.minimum_to_repair(lost, avail)
        pr = {h: rng.integers(0, 256, len(idx) * sc, dtype=np.uint8) for h, idx in info}
        assert c.repair(lost, pr, chunk) == o.repair(lost, pr, chunk), (cfg, sc, lost)


@pytest.mark.parametrize("cfg", [(4, 2, 5), (10, 4, 13), (9, 3, 11)])
@pytest.mark.parametrize("sc,piece,streams", [(8, 0, 0), (1000, 256, 2), (4096 + 8, 1024, 3),
                                              (3 * 2048 + 40, 8, 4), (5000, 0, 1)])
def test_encode_host_pipelined_matches_oracle(oracle_mod, torch_cuda, cfg, sc, piece, streams):
    """Host-streaming encode: pieces of every sub-chunk through 2D copies and several
    streams, ragged last piece; parity identical to the oracle's encode."""
    import torch
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    chunk = c.sub_chunk_no * sc
    data = rand_bytes(sc + piece, k * chunk)
    ref = o.encode_array(data)
    assert ref.shape[1] == chunk
    hs = torch.from_numpy(ref[:k].copy()).pin_memory()
    hp = torch.zeros((m, chunk), dtype=torch.uint8).pin_memory()
    c.encode_host_pipelined([hs[i] for i in range(k)], [hp[j] for j in range(m)], chunk, 0, piece, streams)
    assert np.array_equal(hp.numpy(), ref[k:]), (cfg, sc, piece, streams)
    # pageable numpy buffers take the same path
    dn = [ref[i].copy() for i in range(k)]
    pn = [np.zeros(chunk, np.uint8) for _ in range(m)]
    c.encode_host_pipelined(dn, pn, chunk, 0, piece, streams)
    assert all(np.array_equal(pn[j], ref[k + j]) for j in range(m))


@pytest.mark.parametrize("cfg", [(4, 2, 5), (9, 3, 11), (10, 4, 13), (6, 3, 8)])
def test_repair_device_full_chunks_matches_oracle(oracle_mod, torch_cuda, cfg, exec_mode):
    """Repair straight from whole helper chunks in HBM (no gather): same bytes as the
    oracle's repair on the gathered beta sub-chunks, for codewords and random chunks."""
    torch = torch_cuda
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    sc = 16 * 40 + 6
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc + k)
    code_chunks = c.encode_array(rand_bytes(k, k * chunk))
    for chunks in (code_chunks, rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)):
        dev = torch.from_numpy(np.ascontiguousarray(chunks)).cuda()
        for lost in sorted({0, k - 1, c.n - 1}):
            avail = [i for i in range(c.n) if i != lost]
            info = c.minimum_to_repair(lost, avail)
            out = torch.zeros(chunk, dtype=torch.uint8, device="cuda")
            c.repair_device_full_chunks(lost, [h for h, _ in info], [dev[h] for h, _ in info], chunk, out)
            torch.cuda.synchronize()
            pd = {h: np.concatenate([chunks[h][z * sc:(z + 1) * sc] for z in idx]) for h, idx in info}
            assert out.cpu().numpy().tobytes() == o.repair(lost, pd, chunk), (cfg, lost)


@pytest.mark.parametrize("cfg", [(4, 2, 5), (10, 4, 13), (9, 3, 11), (6, 3, 8), (5, 3, 6)])
@pytest.mark.parametrize("sc,n", [(32, 4), (2, 300), (32, 301), (320, 37), (16 * 70 + 6, 9), (4096, 5), (4104, 6)])
def test_encode_device_batch_small_stripes(oracle_mod, torch_cuda, cfg, sc, n):
    """Batched small stripes: one launch per plan level for the whole batch (grid.y =
    stripe, device pointer table); every stripe's parity equals the oracle's."""
    torch = torch_cuda
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    chunk = c.sub_chunk_no * sc
    refs = [o.encode_array(rand_bytes(100 * s + sc, k * chunk)) for s in range(n)]
    data = torch.from_numpy(np.concatenate([r[:k] for r in refs])).cuda()
    par = torch.zeros((n * m, chunk), dtype=torch.uint8, device="cuda")
    c.encode_device_batch([data[i] for i in range(n * k)], [par[i] for i in range(n * m)], n, chunk)
    torch.cuda.synchronize()
    if k * chunk <= 4 << 20:  # small stripes batch; larger ones keep the per-stripe kernels
        # uniform strides + a bit-sliced kernel + sub-chunks >= half a tile: one
        # bit-sliced launch; otherwise one staged launch per plan level
        assert last_encode_path() == "staged-batch" or last_encode_path().startswith("bitsliced-batch")
        if (k, m) in ((4, 2), (8, 4), (9, 3), (6, 3)) and sc % 8 == 0 and sc >= 1024:
            assert last_encode_path().startswith("bitsliced-batch"), last_encode_path()
    got = par.cpu().numpy()
    for s in range(n):
        assert np.array_equal(got[s * m:(s + 1) * m], refs[s][k:]), (cfg, sc, n, s)

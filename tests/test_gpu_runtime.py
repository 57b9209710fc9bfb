"""GPU runtime behaviour of the C ABI (include/clay.h): concurrency, the device buffer
pool, graph capture and very large batches.  Every result is compared with the oracle.

The reference's ClayCode is immutable and freely shareable across threads (lib.rs:58);
the ABI promises the same: no process-wide lock, any thread, any stream."""
import threading

import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode

pytestmark = pytest.mark.gpu


def rand_bytes(seed, n):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def _stripe(o, k, chunk, seed):
    return o.encode_array(rand_bytes(seed, k * chunk))


def test_threads_and_streams_interleaved(oracle_mod, torch_cuda):
    """2 host threads x 2 streams each, interleaving device encode, 4-erasure decode and
    repair of (10,4,13) stripes, all in flight together; every output bit-exact."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    sc = 4104  # ragged tiles (sc % 16 == 8)
    chunk = c.sub_chunk_no * sc
    refs = [_stripe(o, 10, chunk, 7000 + i) for i in range(4)]
    er = [0, 4, 8, 12]
    lost = 2
    info = c.minimum_to_repair(lost, [i for i in range(14) if i != lost])
    errors = []

    def worker(t):
        try:
            streams = [torch.cuda.Stream() for _ in range(2)]
            jobs = []
            for it in range(6):
                st = streams[it % 2]
                ref = refs[(t * 2 + it) % 4]
                with torch.cuda.stream(st):
                    full = torch.from_numpy(ref).cuda(non_blocking=False)
                    par = torch.zeros((4, chunk), dtype=torch.uint8, device="cuda")
                    c.encode_device([full[i] for i in range(10)], [par[i] for i in range(4)], chunk, 0,
                                    st.cuda_stream)
                    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
                    c.decode_device([None if i in er else full[i] for i in range(14)], er,
                                    [outs[i] if i in er else None for i in range(14)], chunk, 0, st.cuda_stream)
                    rep = torch.zeros(chunk, dtype=torch.uint8, device="cuda")
                    c.repair_device_full_chunks(lost, [h for h, _ in info], [full[h] for h, _ in info], chunk, rep,
                                                0, st.cuda_stream)
                jobs.append((st, ref, par, outs, rep))
            for st, ref, par, outs, rep in jobs:
                st.synchronize()
                assert np.array_equal(par.cpu().numpy(), ref[10:]), "encode"
                for e in er:
                    assert np.array_equal(outs[e].cpu().numpy(), ref[e]), ("decode", e)
                assert np.array_equal(rep.cpu().numpy(), ref[lost]), "repair"
        except Exception as ex:  # noqa: BLE001 -- reported by the main thread
            errors.append((t, repr(ex)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


def test_host_api_concurrent_threads(oracle_mod, torch_cuda):
    """Host-buffer encode / decode from 3 threads at once (each call takes its own pooled
    stream and staging buffers)."""
    c, o = ClayCode(9, 3, 11), oracle_mod.OracleClay(9, 3, 11)
    datas = [bytes(rand_bytes(8100 + t, 9 * 81 * 2 * 37 + t)) for t in range(3)]
    refs = [o.encode(d) for d in datas]
    errors = []

    def worker(t):
        try:
            for _ in range(4):
                got = c.encode(datas[t])
                assert got == refs[t]
                av = {i: got[i] for i in range(12) if i not in (1, 10)}
                assert c.decode(av, [1, 10]) == o.decode(av, [1, 10])
        except Exception as ex:  # noqa: BLE001
            errors.append((t, repr(ex)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


# (round 6: every 2-4 erasure pattern of (10,4,13) streams in auto, so the grouped executor's
# workspace is exercised under exec mode "grouped")
@pytest.mark.parametrize("er,path,mode", [([1, 2, 5, 6], "grouped", "grouped"), ([1, 2, 5, 6], "stream-fused2", "auto"),
                                          ([0, 4, 8, 12], "stream-fused2", "auto")])
def test_workspace_pool_reused_across_streams(oracle_mod, torch_cuda, er, path, mode):
    prev = clay_amd.set_exec_mode(mode)
    try:
        _workspace_pool_reuse(oracle_mod, torch_cuda, er, path)
    finally:
        clay_amd.set_exec_mode(prev)


def _workspace_pool_reuse(oracle_mod, torch_cuda, er, path):
    """Decodes on 8 distinct, short-lived streams one after another reuse the pooled
    workspace (the grouped executor's U workspace; the fused decode v2 needs none): the pool
    does not grow per stream (it grew by one workspace per stream handle before the pool
    existed)."""
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    sc = 1024
    chunk = c.sub_chunk_no * sc
    ref = _stripe(o, 10, chunk, 99)
    full = torch.from_numpy(ref).cuda()
    clay_amd.release_workspace(0)
    sizes = []
    for i in range(8):
        st = torch.cuda.Stream()
        outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
        c.decode_device([None if j in er else full[j] for j in range(14)], er,
                        [outs[j] if j in er else None for j in range(14)], chunk, 0, st.cuda_stream)
        st.synchronize()
        assert clay_amd.last_exec_path() == path
        for e in er:
            assert np.array_equal(outs[e].cpu().numpy(), ref[e])
        sizes.append(clay_amd.workspace_bytes(0))
        del st
    # one U workspace (q t = 16 nodes); the fused decode v2 takes none
    assert sizes[0] >= 16 * chunk if path == "grouped" else sizes[0] == 0
    assert sizes[-1] == sizes[0], sizes
    clay_amd.release_workspace(0)
    assert clay_amd.workspace_bytes(0) == 0


def test_reserve_then_no_growth(oracle_mod, torch_cuda):
    """clay_reserve_workspace leaves an idle workspace any stream can take."""
    torch = torch_cuda
    c, o = ClayCode(4, 2, 5), oracle_mod.OracleClay(4, 2, 5)
    chunk = c.sub_chunk_no * 4096
    clay_amd.release_workspace(0)
    c.reserve_workspace(chunk)
    reserved = clay_amd.workspace_bytes(0)
    assert reserved >= c.q * c.t * chunk
    ref = _stripe(o, 4, chunk, 5)
    full = torch.from_numpy(ref).cuda()
    st = torch.cuda.Stream()
    outs = torch.zeros((6, chunk), dtype=torch.uint8, device="cuda")
    c.decode_device([None if j == 0 else full[j] for j in range(6)], [0], [outs[0]] + [None] * 5, chunk, 0,
                    st.cuda_stream)
    st.synchronize()
    assert np.array_equal(outs[0].cpu().numpy(), ref[0])
    assert clay_amd.workspace_bytes(0) == reserved


def test_batch_encode_graph_capture(oracle_mod, torch_cuda):
    """Batched small-stripe encode captured into a HIP graph and replayed on new data:
    the pointer table is uploaded once from pinned memory (no blocking copy, no stream
    sync inside the call), so the call is capturable."""
    torch = torch_cuda
    k, m, d = 4, 2, 5
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    n, chunk = 16, c.sub_chunk_no * 512
    data = torch.zeros((n * k, chunk), dtype=torch.uint8, device="cuda")
    par = torch.zeros((n * m, chunk), dtype=torch.uint8, device="cuda")
    dl, pl = [data[i] for i in range(n * k)], [par[i] for i in range(n * m)]
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):  # warm-up outside capture: plan upload, workspace
        c.encode_device_batch(dl, pl, n, chunk, 0, st.cuda_stream)
    st.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        c.encode_device_batch(dl, pl, n, chunk, 0, torch.cuda.current_stream().cuda_stream)
    for rep in range(2):
        refs = [_stripe(o, k, chunk, 300 + 10 * rep + s) for s in range(n)]
        data.copy_(torch.from_numpy(np.concatenate([r[:k] for r in refs])))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        got = par.cpu().numpy()
        for s in range(n):
            assert np.array_equal(got[s * m:(s + 1) * m], refs[s][k:]), (rep, s)


def test_batch_encode_more_than_grid_y_limit(oracle_mod, torch_cuda):
    """70,000 (4,2,5) 1 KiB-class stripes in one call: split into launch groups of at
    most 65,535 stripes (the grid.y limit); stripes either side of the split match."""
    torch = torch_cuda
    k, m, d = 4, 2, 5
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    n, chunk = 70000, c.sub_chunk_no * 32  # sc 32 -> 256-byte chunks, 1 KiB of data per stripe
    host = rand_bytes(4242, n * k * chunk).reshape(n * k, chunk)
    data = torch.from_numpy(host).cuda()
    par = torch.zeros((n * m, chunk), dtype=torch.uint8, device="cuda")
    c.encode_device_batch([data[i] for i in range(n * k)], [par[i] for i in range(n * m)], n, chunk)
    torch.cuda.synchronize()
    assert clay_amd.last_encode_path() == "staged-batch"
    got = par.cpu().numpy()
    for s in (0, 1, 65534, 65535, 65536, n - 1):
        ref = o.encode_array(host[s * k:(s + 1) * k].reshape(-1))
        assert np.array_equal(got[s * m:(s + 1) * m], ref[k:]), s


@pytest.mark.parametrize("sc,n", [(32, 300), (4104, 5)])
def test_batch_encode_non_affine_pointers(oracle_mod, torch_cuda, sc, n):
    """Stripes whose chunks are NOT rows of one strided buffer (permuted order) take the
    device pointer-table path; a second call with the same buffers reuses the cached
    table.  Affine batches (the other tests) pass base + stride in kernel arguments."""
    torch = torch_cuda
    k, m, d = 6, 3, 8
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    chunk = c.sub_chunk_no * sc
    refs = [_stripe(o, k, chunk, 900 + s) for s in range(n)]
    perm = np.random.default_rng(3).permutation(n)
    data = torch.from_numpy(np.concatenate([refs[s][:k] for s in perm])).cuda()
    par = torch.zeros((n * m, chunk), dtype=torch.uint8, device="cuda")
    slot = {s: j for j, s in enumerate(perm)}  # stripe s lives at data block slot[s]
    dl = [data[slot[s] * k + i] for s in range(n) for i in range(k)]
    pl = [par[slot[s] * m + i] for s in range(n) for i in range(m)]
    for _ in range(2):
        par.zero_()
        c.encode_device_batch(dl, pl, n, chunk)
        torch.cuda.synchronize()
        got = par.cpu().numpy()
        for s in range(n):
            assert np.array_equal(got[slot[s] * m:(slot[s] + 1) * m], refs[s][k:]), s


def test_non_affine_table_across_streams_and_capture(oracle_mod, torch_cuda):
    """A non-affine pointer table first uploaded on stream A is then used on stream B
    (which must wait for A's upload), inside a graph capture on stream C (a private,
    graph-owned upload), and eagerly again after the capture -- every result bit-exact.
    Outputs start as 0xFF so a skipped write shows."""
    torch = torch_cuda
    k, m, d = 6, 3, 8
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    n, sc = 40, 32
    chunk = c.sub_chunk_no * sc
    refs = [_stripe(o, k, chunk, 1300 + s) for s in range(n)]
    perm = np.random.default_rng(5).permutation(n)
    data = torch.from_numpy(np.concatenate([refs[s][:k] for s in perm])).cuda()
    slot = {s: j for j, s in enumerate(perm)}
    pars = [torch.full((n * m, chunk), 0xFF, dtype=torch.uint8, device="cuda") for _ in range(4)]
    dl = [data[slot[s] * k + i] for s in range(n) for i in range(k)]

    def pl(par):
        return [par[slot[s] * m + i] for s in range(n) for i in range(m)]

    def check(par, what):
        got = par.cpu().numpy()
        for s in range(n):
            assert np.array_equal(got[slot[s] * m:(slot[s] + 1) * m], refs[s][k:]), (what, s)

    clay_amd.release_workspace(0)
    sa, sb, sc_, sd = (torch.cuda.Stream() for _ in range(4))
    # A uploads the table for pars[0]'s pointer set; B reuses the same set right away
    c.encode_device_batch(dl, pl(pars[0]), n, chunk, 0, sa.cuda_stream)
    c.encode_device_batch(dl, pl(pars[0]), n, chunk, 0, sb.cuda_stream)
    sb.synchronize()
    sa.synchronize()
    check(pars[0], "A then B")
    # a table first seen inside a capture, then the same pointer set eagerly on D (the capture
    # takes an idle reserved workspace: nothing may be allocated while capturing)
    c.reserve_workspace(n * chunk)  # the batch's U workspace: tn x chunk per stripe
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=sc_):
        c.encode_device_batch(dl, pl(pars[1]), n, chunk, 0, torch.cuda.current_stream().cuda_stream)
    c.encode_device_batch(dl, pl(pars[1]), n, chunk, 0, sd.cuda_stream)
    sd.synchronize()
    check(pars[1], "eager after capture")
    pars[1].fill_(0xFF)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    check(pars[1], "replay")


def test_tile_executor_writes_every_output(oracle_mod, torch_cuda):
    """Decode and repair under the tile-fused executor with outputs pre-filled with 0xFF:
    every destination byte is written (no stale caller bytes survive)."""
    torch = torch_cuda
    prev = clay_amd.set_exec_mode("tile")
    try:
        for (k, m, d), er, lost in (((4, 2, 5), [0], 1), ((6, 3, 8), [1, 7], 0)):
            c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
            n = k + m
            chunk = c.sub_chunk_no * 1024
            ref = _stripe(o, k, chunk, 77 + k)
            full = torch.from_numpy(ref).cuda()
            outs = torch.full((n, chunk), 0xFF, dtype=torch.uint8, device="cuda")
            c.decode_device([None if j in er else full[j] for j in range(n)], er,
                            [outs[j] if j in er else None for j in range(n)], chunk)
            rep = torch.full((chunk,), 0xFF, dtype=torch.uint8, device="cuda")
            info = c.minimum_to_repair(lost, [i for i in range(n) if i != lost])
            c.repair_device_full_chunks(lost, [h for h, _ in info], [full[h] for h, _ in info], chunk, rep)
            torch.cuda.synchronize()
            for e in er:
                assert np.array_equal(outs[e].cpu().numpy(), ref[e]), ((k, m, d), e)
            assert np.array_equal(rep.cpu().numpy(), ref[lost]), ((k, m, d), "repair")
    finally:
        clay_amd.set_exec_mode(prev)


@pytest.mark.parametrize("cfg,sc,n,pad", [((4, 2, 5), 32, 300, 0), ((4, 2, 5), 32, 3, 0), ((10, 4, 13), 40, 9, 64),
                                          ((9, 3, 11), 2, 257, 16), ((6, 3, 8), 4104, 5, 0),
                                          ((10, 4, 13), 2048, 5, 0)])
def test_encode_device_strided(oracle_mod, torch_cuda, cfg, sc, n, pad):
    """clay_encode_device_strided: stripes at fixed strides (node stride = chunk + pad),
    small batches (staged batch), n < 4 and > 4 MiB stripes (per-stripe kernels)."""
    torch = torch_cuda
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    chunk = c.sub_chunk_no * sc
    row = chunk + pad
    refs = [_stripe(o, k, chunk, 1300 + s) for s in range(n)]
    host = np.zeros((n, k, row), np.uint8)
    for s in range(n):
        host[s, :, :chunk] = refs[s][:k]
    data = torch.from_numpy(host).cuda()
    par = torch.zeros((n, m, row), dtype=torch.uint8, device="cuda")
    c.encode_device_strided(data, par, n, chunk, row, k * row, row, m * row)
    torch.cuda.synchronize()
    got = par.cpu().numpy()
    for s in range(n):
        assert np.array_equal(got[s, :, :chunk], refs[s][k:]), s
        assert not got[s, :, chunk:].any()


# ---------------------------------------------------------------------------
# Y-grouped ("Option C") layout, SURVEY.md §8f item 3
# ---------------------------------------------------------------------------
def ygroup_order(c, y):
    """docs/clay-practical-implementation.md:453-490 construct_groups, restated with the
    crate's MSB-first digits (coords.rs:30-40): blocks x of layers with digit_y == x."""
    q, t, alpha = c.q, c.t, c.sub_chunk_no
    digit = lambda z: (z // q ** (t - 1 - y)) % q  # noqa: E731
    return [z for x in range(q) for z in range(alpha) if digit(z) == x]


@pytest.mark.parametrize("cfg,sc", [((10, 4, 13), 100), ((9, 3, 11), 4098), ((4, 2, 5), 9000), ((6, 3, 8), 2)])
def test_ygroup_layout_and_repair(oracle_mod, torch_cuda, cfg, sc):
    """Regroup = the restated permutation; inverse restores the chunk; repairing node
    (y, x) from each helper's contiguous block x of group y equals the oracle's repair."""
    torch = torch_cuda
    k, m, d = cfg
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    chunk = c.sub_chunk_no * sc
    ref = _stripe(o, k, chunk, 4242 + sc)
    full = torch.from_numpy(ref).cuda()
    for lost in range(c.n):
        li = lost if lost < k else lost + c.nu
        y, x = divmod(li, c.q)
        info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
        order = ygroup_order(c, y)
        beta = c.beta
        assert order[x * beta:(x + 1) * beta] == list(info[0][1])  # block x = repair indices
        groups = torch.empty((c.n, chunk), dtype=torch.uint8, device="cuda")
        for h, _ in info:
            c.chunk_to_ygroup(y, full[h], groups[h], chunk)
        torch.cuda.synchronize()
        for h, _ in info:
            want = ref[h].reshape(c.sub_chunk_no, sc)[order].reshape(-1)
            assert np.array_equal(groups[h].cpu().numpy(), want), (lost, h)
        out = torch.zeros(chunk, dtype=torch.uint8, device="cuda")
        c.repair_device(lost, [h for h, _ in info], [groups[h][x * beta * sc:(x + 1) * beta * sc] for h, _ in info],
                        chunk, out)
        back = torch.zeros(chunk, dtype=torch.uint8, device="cuda")
        h0 = info[0][0]
        c.ygroup_to_chunk(y, groups[h0], back, chunk)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), ref[lost]), lost
        assert np.array_equal(back.cpu().numpy(), ref[h0])


def test_capture_arena_reclaimed(oracle_mod, torch_cuda):
    """Pointer tables of batch calls inside stream captures come from a fixed per-device
    arena (no allocation while capturing).  Captures of a 300-stripe non-affine batch fill it
    after about a dozen graphs; clay_release_captured, once those graphs are destroyed,
    gives it back, and later captures replay bit-exact."""
    torch = torch_cuda
    k, m, d = 6, 3, 8
    c, o = ClayCode(k, m, d), oracle_mod.OracleClay(k, m, d)
    n, sc = 300, 32
    chunk = c.sub_chunk_no * sc
    refs = [_stripe(o, k, chunk, 2100 + s) for s in range(n)]
    perm = np.random.default_rng(11).permutation(n)
    slot = {s: j for j, s in enumerate(perm)}
    data = torch.from_numpy(np.concatenate([refs[s][:k] for s in perm])).cuda()
    par = torch.full((n * m, chunk), 0xFF, dtype=torch.uint8, device="cuda")
    dl = [data[slot[s] * k + i] for s in range(n) for i in range(k)]
    pl = [par[slot[s] * m + i] for s in range(n) for i in range(m)]
    st = torch.cuda.Stream()
    clay_amd.release_captured(0)
    c.reserve_workspace(n * chunk)
    c.encode_device_batch(dl, pl, n, chunk, 0, st.cuda_stream)  # plan upload outside capture
    st.synchronize()

    def capture():
        c.reserve_workspace(n * chunk)  # each captured call keeps its workspace: one idle lease per capture
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            c.encode_device_batch(dl, pl, n, chunk, 0, torch.cuda.current_stream().cuda_stream)
        return g

    graphs, failed = [], None
    for _ in range(20):
        try:
            graphs.append(capture())
        except clay_amd.DeviceError as ex:
            failed = str(ex)
            break
    assert failed is not None and "arena" in failed, (len(graphs), failed)
    assert 8 <= len(graphs) <= 14, len(graphs)
    par.fill_(0xFF)
    torch.cuda.synchronize()
    graphs[-1].replay()
    torch.cuda.synchronize()
    got = par.cpu().numpy()
    for s in range(n):
        assert np.array_equal(got[slot[s] * m:(slot[s] + 1) * m], refs[s][k:]), ("before release", s)
    del graphs
    clay_amd.release_captured(0)
    for rep in range(3):  # more captures than the arena held before: each one reclaimed
        g = capture()
        par.fill_(0xFF)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        got = par.cpu().numpy()
        for s in range(n):
            assert np.array_equal(got[slot[s] * m:(slot[s] + 1) * m], refs[s][k:]), (rep, s)
        del g
        clay_amd.release_captured(0)


@pytest.mark.parametrize("mode,path,er,er2", [("grouped", "grouped", [0, 4, 8, 12], [1, 5, 9, 13]),
                                              ("auto", "stream-fused2", [0, 4, 8, 12], [1, 5, 9, 13]),
                                              ("auto", "stream-local256", [0, 4], [1, 5])])
def test_decode_graph_capture_after_prepare(oracle_mod, torch_cuda, mode, path, er, er2):
    """A (10,4,13) decode inside a stream capture, on the grouped executor (its U workspace lease
    covered by the reserved workspace), on the fused decode v2 and on the local decode on 256-byte
    runs (no workspace): one eager call of the pattern prepared its tables, so the capture
    allocates nothing (the pool does not grow) and replays bit-exact on new data.  A pattern never
    run before fails inside the capture with a clear error instead of invalidating it."""
    prev = clay_amd.set_exec_mode(mode)
    try:
        _decode_graph_capture(oracle_mod, torch_cuda, path, er, er2)
    finally:
        clay_amd.set_exec_mode(prev)


def _decode_graph_capture(oracle_mod, torch_cuda, path, er, er2):
    torch = torch_cuda
    c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
    sc = 1024
    chunk = c.sub_chunk_no * sc
    st = torch.cuda.Stream()
    clay_amd.release_captured(0)
    clay_amd.release_workspace(0)
    c.reserve_workspace(chunk)
    reserved = clay_amd.workspace_bytes(0)
    assert reserved >= c.q * c.t * chunk
    full = torch.from_numpy(_stripe(o, 10, chunk, 77)).cuda()
    outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
    args = ([None if j in er else full[j] for j in range(14)], er, [outs[j] if j in er else None for j in range(14)])
    c.decode_device(*args, chunk, 0, st.cuda_stream)  # prepares the pattern's tables
    st.synchronize()
    assert clay_amd.last_exec_path() == path
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        c.decode_device(*args, chunk, 0, torch.cuda.current_stream().cuda_stream)
    assert clay_amd.workspace_bytes(0) == reserved
    for rep in range(2):
        ref = _stripe(o, 10, chunk, 780 + rep)
        full.copy_(torch.from_numpy(ref))
        outs.fill_(0xA5)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        for e in er:
            assert np.array_equal(outs[e].cpu().numpy(), ref[e]), (rep, e)
    g2 = torch.cuda.CUDAGraph()
    with pytest.raises(clay_amd.DeviceError, match="not prepared"):
        with torch.cuda.graph(g2, stream=st):
            c.decode_device([None if j in er2 else full[j] for j in range(14)], er2,
                            [outs[j] if j in er2 else None for j in range(14)], chunk, 0,
                            torch.cuda.current_stream().cuda_stream)
    del g, g2
    torch.cuda.synchronize()
    clay_amd.release_captured(0)


def test_release_captured_refused_while_capture_open(oracle_mod, torch_cuda):
    """clay_release_captured while another thread holds a capture open that took a pooled
    workspace (grouped-executor decode): refused, and the workspace stays with the graph (the
    pool does not hand it out); once the capture ended, the graph replayed, its stream was
    synchronised and the graph destroyed, the same call succeeds."""
    torch = torch_cuda
    prev = clay_amd.set_exec_mode("grouped")
    try:
        c, o = ClayCode(10, 4, 13), oracle_mod.OracleClay(10, 4, 13)
        sc = 256
        chunk = c.sub_chunk_no * sc
        er = [0, 4, 8, 12]
        st = torch.cuda.Stream()
        clay_amd.release_captured(0)
        clay_amd.release_workspace(0)
        c.reserve_workspace(chunk)
        ref = _stripe(o, 10, chunk, 91)
        full = torch.from_numpy(ref).cuda()
        outs = torch.zeros((14, chunk), dtype=torch.uint8, device="cuda")
        args = ([None if j in er else full[j] for j in range(14)], er,
                [outs[j] if j in er else None for j in range(14)])
        c.decode_device(*args, chunk, 0, st.cuda_stream)  # prepares the plan outside the capture
        st.synchronize()
        inside, release_now, done = threading.Event(), threading.Event(), threading.Event()
        box = {}

        def capturer():
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    c.decode_device(*args, chunk, 0, torch.cuda.current_stream().cuda_stream)
                    inside.set()
                    release_now.wait(60)  # the capture stays open until the main thread tried
                box["g"] = g
            except BaseException as ex:  # noqa: BLE001
                box["err"] = ex
                inside.set()
            finally:
                done.set()

        th = threading.Thread(target=capturer)
        th.start()
        assert inside.wait(60)
        refused = None
        try:
            clay_amd.release_captured(0)
        except clay_amd.DeviceError as ex:
            refused = str(ex)
        release_now.set()
        th.join(120)
        assert done.is_set() and "err" not in box, box.get("err")
        assert refused is not None and "pooled workspace" in refused, refused
        outs.fill_(0)
        torch.cuda.synchronize()
        box["g"].replay()
        torch.cuda.synchronize()
        for e in er:
            assert np.array_equal(outs[e].cpu().numpy(), ref[e]), e
        del box["g"]
        torch.cuda.synchronize()
        clay_amd.release_captured(0)  # capture closed, replays done, graph destroyed: accepted
    finally:
        clay_amd.set_exec_mode(prev)

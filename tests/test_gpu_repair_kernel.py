"""GPU parity of the bit-sliced single-launch repair kernel (repair_kernel.hpp) against the
oracle: every lost node of the q = m codes it is instantiated for, helper data as gathered beta
sub-chunks (clay_repair_device) and as whole chunks (clay_repair_device_full_chunks), on random
(non-codeword) helper bytes, sub-chunks of every alignment, partial last tiles.
Reference: repair.rs:140-421 (phases 1-3), minimum_to_repair repair.rs:61-126."""
import numpy as np
import pytest

import clay_amd
from clay_amd import ClayCode

pytestmark = pytest.mark.gpu


# codes with a streaming kernel (k_bs_repair_stream; exec mode "stream" runs it for sub-chunks of
# at least 16 bytes, partial last tiles included)
STREAM_CODES = {(9, 3, 11), (10, 4, 13)}


def expect_path(cfg, sc):
    return "bs-repair-stream" if cfg in STREAM_CODES and sc >= 16 else "bs-repair"


@pytest.fixture
def stream_exec():
    prev = clay_amd.set_exec_mode("stream")
    yield
    clay_amd.set_exec_mode(prev)


@pytest.mark.parametrize("cfg", [(9, 3, 11), (10, 4, 13), (4, 2, 5)])
@pytest.mark.parametrize("sc", [2, 16, 37, 288 + 2, 512, 1000, 4096 + 6])
def test_bs_repair_every_node_random_helpers(oracle_mod, torch_cuda, stream_exec, cfg, sc):
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    rng = np.random.default_rng(sc * 31 + cfg[0])
    full = rng.integers(0, 256, (c.n, chunk), dtype=np.uint8)  # random: not a codeword
    fd = torch.from_numpy(full).cuda()
    for lost in range(c.n):
        info = c.minimum_to_repair(lost, [i for i in range(c.n) if i != lost])
        helpers = [h for h, _ in info]
        hd = {h: np.concatenate([full[h][z * sc:(z + 1) * sc] for z in idx]) for h, idx in info}
        ref = np.frombuffer(o.repair(lost, hd, chunk), dtype=np.uint8)
        hb = torch.from_numpy(np.stack([hd[h] for h in helpers])).cuda()
        out = torch.full((chunk,), 0xA5, dtype=torch.uint8, device="cuda")
        c.repair_device(lost, helpers, [hb[i] for i in range(len(helpers))], chunk, out)
        torch.cuda.synchronize()
        assert clay_amd.last_exec_path() == expect_path(cfg, sc), clay_amd.last_exec_path()
        assert np.array_equal(out.cpu().numpy(), ref), (cfg, sc, lost, "gathered")
        out.fill_(0x5A)
        c.repair_device_full_chunks(lost, helpers, [fd[h] for h in helpers], chunk, out)
        torch.cuda.synchronize()
        assert clay_amd.last_exec_path() == expect_path(cfg, sc)
        assert np.array_equal(out.cpu().numpy(), ref), (cfg, sc, lost, "full chunks")


def test_bs_repair_matches_grouped_executor(oracle_mod, torch_cuda):
    """(9,3,11) at sc = 3,314,018 / 64 (2 mod 8 like the BASELINE chunk): the kernel and the
    grouped plan executor produce the same bytes for node 0 and node 11."""
    torch = torch_cuda
    c = ClayCode(9, 3, 11)
    sc = 3314018 // 64 + 8 * 0
    sc -= sc % 8
    sc += 2
    chunk = c.sub_chunk_no * sc
    full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda")
    prev = clay_amd.set_exec_mode("stream")
    try:
        for lost in (0, 11):
            helpers = [i for i in range(c.n) if i != lost]
            a = torch.empty(chunk, dtype=torch.uint8, device="cuda")
            b = torch.empty(chunk, dtype=torch.uint8, device="cuda")
            clay_amd.set_exec_mode("stream")
            c.repair_device_full_chunks(lost, helpers, [full[h] for h in helpers], chunk, a)
            assert clay_amd.last_exec_path() == "bs-repair-stream"
            clay_amd.set_exec_mode("grouped")
            c.repair_device_full_chunks(lost, helpers, [full[h] for h in helpers], chunk, b)
            assert clay_amd.last_exec_path() == "grouped"
            torch.cuda.synchronize()
            assert torch.equal(a, b), lost
    finally:
        clay_amd.set_exec_mode(prev)


@pytest.mark.parametrize("cfg,sc", [((9, 3, 11), 512 * 256 * 3 + 37), ((10, 4, 13), 256 * 256 * 3 + 8)])
def test_bs_repair_stream_many_tiles(oracle_mod, torch_cuda, cfg, sc):
    """Several tiles per workgroup (the LDS ring wraps across tiles and within a tile) plus a
    partial last tile: auto mode picks the streaming kernel; every lost node equals the grouped plan
    executor (gathered helpers and whole chunks), two nodes are checked against the oracle."""
    torch = torch_cuda
    c, o = ClayCode(*cfg), oracle_mod.OracleClay(*cfg)
    chunk = c.sub_chunk_no * sc
    full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda")
    prev = clay_amd.set_exec_mode("auto")
    try:
        for lost in range(c.n):
            helpers = [i for i in range(c.n) if i != lost]
            a = torch.full((chunk,), 0xA5, dtype=torch.uint8, device="cuda")
            b = torch.full((chunk,), 0x5A, dtype=torch.uint8, device="cuda")
            clay_amd.set_exec_mode("auto")
            c.repair_device_full_chunks(lost, helpers, [full[h] for h in helpers], chunk, a)
            assert clay_amd.last_exec_path() == "bs-repair-stream"
            assert clay_amd.last_launch_count() == 1  # the partial last tile is in the same launch
            clay_amd.set_exec_mode("grouped")
            c.repair_device_full_chunks(lost, helpers, [full[h] for h in helpers], chunk, b)
            torch.cuda.synchronize()
            assert torch.equal(a, b), (cfg, lost, "full chunks")
            if lost in (0, c.n - 1):
                info = c.minimum_to_repair(lost, helpers)
                fh = full.cpu().numpy()
                hd = {h: np.concatenate([fh[h][z * sc:(z + 1) * sc] for z in idx]) for h, idx in info}
                ref = np.frombuffer(o.repair(lost, hd, chunk), dtype=np.uint8)
                hb = torch.from_numpy(np.stack([hd[h] for h, _ in info])).cuda()
                clay_amd.set_exec_mode("auto")
                a.fill_(0)
                c.repair_device(lost, [h for h, _ in info], [hb[i] for i in range(len(info))], chunk, a)
                torch.cuda.synchronize()
                assert clay_amd.last_exec_path() == "bs-repair-stream"
                assert np.array_equal(a.cpu().numpy(), ref), (cfg, lost, "gathered vs oracle")
                del hb
    finally:
        clay_amd.set_exec_mode(prev)

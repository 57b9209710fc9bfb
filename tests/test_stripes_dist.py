"""Multi-process stripe sharding on CPU (gloo, world_size 2): the N>1 path of bench.py.

Each rank takes its block of global stripe ids, encodes them (here with the oracle --
test infrastructure; on the GPU box ranks run the HIP kernels), and the union of the
ranks' parity equals the single-process result.  Only the timing max is reduced."""
import os
import socket

import numpy as np
import pytest

from clay_amd.stripes import aggregate_rate, assign_stripes


def test_assign_stripes_partitions():
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            got = [assign_stripes(n, w, r) for r in range(w)]
            flat = [s for g in got for s in g]
            assert flat == list(range(n))
            assert max(map(len, got)) - min(map(len, got)) <= 1
    assert aggregate_rate([10, 10], [1.0, 2.0]) == 10.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_stripes, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    from clay_amd.stripes import assign_stripes, reduce_max_time
    from oracle import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    code = oracle.OracleClay(10, 4, 13)
    for s in assign_stripes(n_stripes, world, rank):
        data = np.random.default_rng(s).integers(0, 256, 10 * 256 * 2 * 4, dtype=np.uint8)
        np.save(os.path.join(out_dir, f"par_{s}.npy"), code.encode_array(data)[10:])
    t = reduce_max_time(0.5 + rank)
    np.save(os.path.join(out_dir, f"t_{rank}.npy"), np.array([t]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_stripe_sharding(tmp_path, oracle_mod):
    import torch.multiprocessing as mp
    n_stripes, world = 5, 2
    mp.spawn(_worker, args=(world, _free_port(), n_stripes, str(tmp_path)), nprocs=world, join=True)
    code = oracle_mod.OracleClay(10, 4, 13)
    for s in range(n_stripes):
        data = np.random.default_rng(s).integers(0, 256, 10 * 256 * 2 * 4, dtype=np.uint8)
        assert np.array_equal(np.load(tmp_path / f"par_{s}.npy"), code.encode_array(data)[10:])
    for r in range(world):
        assert float(np.load(tmp_path / f"t_{r}.npy")[0]) == pytest.approx(1.5)

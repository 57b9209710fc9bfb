"""Stripe-parallel scheduling across GPUs (one process per GPU).

Clay stripes are independent codewords (encode.rs:30-80 works on one data
buffer; nothing crosses stripes), and inside a stripe every byte offset of the
sub-chunks is an independent codeword.  Multi-GPU encode therefore needs no
data-path collective: global stripe ids are dealt to ranks, each rank encodes its
own stripes on its own device, and only timing metadata is reduced.
"""
from __future__ import annotations

from typing import List, Sequence


def assign_stripes(n_stripes: int, world: int, rank: int) -> List[int]:
    """Contiguous block assignment of global stripe ids to `rank` (balanced to +-1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_stripes, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def aggregate_rate(bytes_per_rank: Sequence[int], times: Sequence[float]) -> float:
    """Whole-job throughput: all bytes / the slowest rank's time (weak-scaling convention)."""
    t = max(times)
    return float(sum(bytes_per_rank)) / t if t > 0 else 0.0


def reduce_max_time(elapsed: float) -> float:
    """MAX over ranks of a wall time (timing plumbing only; identity when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(elapsed)
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

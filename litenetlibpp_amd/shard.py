"""Multi-GPU layout of a batch: one process per GPU, contiguous datagram
ranges, no collective on the data path.

The only collectives used by the benchmark are a barrier and a MAX over the
per-rank times (timing, not data).  Works with any torch.distributed backend
("nccl" = RCCL on the GPU box, "gloo" in the CPU tests).  The reductions run
whenever a process group is initialised -- also at world size 1, which is how
``bench.py --force-dist`` exercises the RCCL branch on one GPU.
"""
from __future__ import annotations


def shard_range(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """[start, start + count) of the datagrams owned by `rank`: contiguous
    blocks of ceil(n_total / world), the last one possibly shorter/empty."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    per = -(-n_total // world)
    start = min(rank * per, n_total)
    return start, min(per, n_total - start)


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a per-rank scalar (the job's time is its slowest rank's)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(value: float, device=None) -> list[float]:
    """Every rank's scalar, in rank order (reporting only)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def sum_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item())

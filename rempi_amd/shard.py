"""Multi-GPU layout of the CDC batch path: rank traces are independent, so each GPU takes one
contiguous block of the job's ranks and exchanges nothing on the data path.  Rank r of an
R-rank job goes to GPU floor(r * G / R); a GPU walks its block in batches that fit HBM.  The
only collective is the end-of-run reduction of counters (sum) and elapsed time (max), over
RCCL on the GPU box (`nccl` backend) and gloo in the CPU tests.  bench.py uses these helpers."""
from __future__ import annotations

import numpy as np


def gpu_of_rank(rank: int, world: int, n_gpus: int) -> int:
    """floor(rank * G / R): the GPU that processes `rank`'s trace."""
    return rank * n_gpus // world


def block(world: int, n_gpus: int, gpu: int) -> tuple[int, int]:
    """(first rank, rank count) of GPU `gpu`: the ranks r with floor(r * G / R) == gpu, i.e.
    [ceil(gpu * R / G), ceil((gpu + 1) * R / G)).  The blocks of all GPUs partition [0, R)."""
    if n_gpus < 1 or not 0 <= gpu < n_gpus or world < 1:
        raise ValueError("bad shard request")
    lo = -(-gpu * world // n_gpus)
    hi = -(-(gpu + 1) * world // n_gpus)
    return lo, hi - lo


def check_cover(world: int, n_gpus: int) -> None:
    """Every rank of the job lies in exactly one GPU's block, and in the block of its GPU."""
    nxt = 0
    for g in range(n_gpus):
        first, n = block(world, n_gpus, g)
        if first != nxt:
            raise AssertionError(f"GPU {g} starts at rank {first}, expected {nxt}")
        if n and (gpu_of_rank(first, world, n_gpus) != g or gpu_of_rank(first + n - 1, world, n_gpus) != g):
            raise AssertionError(f"GPU {g} holds ranks of another GPU")
        nxt = first + n
    if nxt != world:
        raise AssertionError(f"blocks end at rank {nxt}, job has {world}")


def batches(first: int, count: int, per_batch: int) -> list[tuple[int, int]]:
    """Split a GPU's block into the fewest batches of at most `per_batch` resident rank traces,
    sized evenly (e.g. 128 ranks at 96 per batch -> 64 + 64)."""
    if per_batch < 1:
        raise ValueError("per_batch must be positive")
    if count <= 0:
        return []
    nb = -(-count // per_batch)
    out, at = [], first
    for i in range(nb):
        n = count // nb + (1 if i < count % nb else 0)
        out.append((at, n))
        at += n
    return out


def lane_sizes(count: int, streams: int) -> list[int]:
    """Split a batch's ranks over `streams` in-flight lanes (one HIP stream each)."""
    s = max(1, min(streams, count))
    return [count // s + (1 if i < count % s else 0) for i in range(s)]


def reduce_counters(counters, elapsed: float, dist=None, device="cpu"):
    """Sum the counter vector (whole numbers: records, bytes, ranks; kept and reduced as 64-bit
    integers, so sums stay exact past 2^53) and take the max elapsed time over all processes."""
    c = np.asarray(counters, dtype=np.int64)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return c, float(elapsed)
    import torch

    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = torch.tensor(c, dtype=torch.int64, device=device)
    dist.all_reduce(v)
    return v.cpu().numpy(), float(t.item())

"""Multi-GPU layout of the CDC batch path: rank traces are independent, so
GPUs take contiguous blocks of ranks and exchange nothing on the data path.  The only
collective is the end-of-run reduction of counters (sum) and elapsed time (max), over RCCL
on the GPU box (`nccl` backend) and gloo in the CPU tests.  bench.py uses these helpers."""
from __future__ import annotations

import numpy as np


def shard(world: int, n_gpus: int, gpu: int, per_gpu: int) -> tuple[int, int]:
    """First rank and rank count of GPU `gpu`: block [gpu*per_gpu, (gpu+1)*per_gpu) of the
    job's ranks (wrapping past `world`, so a weak-scaling run of any size keeps per-GPU work
    fixed)."""
    if n_gpus < 1 or not 0 <= gpu < n_gpus or per_gpu < 1 or world < 1:
        raise ValueError("bad shard request")
    return (gpu * per_gpu) % world, per_gpu


def lane_sizes(count: int, streams: int) -> list[int]:
    """Split a GPU's ranks over `streams` in-flight batches (one HIP stream each)."""
    s = max(1, min(streams, count))
    return [count // s + (1 if i < count % s else 0) for i in range(s)]


def reduce_counters(counters, elapsed: float, dist=None, device="cpu"):
    """Sum the counter vector and take the max elapsed time over all processes."""
    c = np.asarray(counters, dtype=np.float64)
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return c, float(elapsed)
    import torch

    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = torch.tensor(c, dtype=torch.float64, device=device)
    dist.all_reduce(v)
    return v.cpu().numpy(), float(t.item())

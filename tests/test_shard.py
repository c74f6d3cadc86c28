"""The N>1 path of bench.py on CPU: ranks shard into disjoint contiguous blocks with no
data-path exchange, and the end-of-run reduction (sum of counters, max of elapsed time)
over a world_size-2 gloo group equals the single-process totals."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import rempi_amd
from rempi_amd import shard


def test_shard_blocks_are_disjoint_and_cover():
    world, per = 64, 8
    seen = []
    for g in range(8):
        first, n = shard.shard(world, 8, g, per)
        seen += list(range(first, first + n))
    assert sorted(seen) == list(range(64))
    assert shard.lane_sizes(10, 4) == [3, 3, 2, 2]
    assert shard.lane_sizes(3, 8) == [1, 1, 1]
    with pytest.raises(ValueError):
        shard.shard(64, 2, 2, 8)


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    p = rempi_amd.default_gen_params(world_size=16, events_per_rank=3000)
    first, n = shard.shard(16, ws, rank, 2)
    recs = comp = 0
    for r in range(first, first + n):  # each process encodes only its own ranks
        h = rempi_amd.generate_host(p, r)
        recs += h.shape[0]
        comp += len(O.encode(h, 4096)[0])
    c, t = shard.reduce_counters([recs, comp, 0], 1.0 + rank, dist)
    q.put((rank, c.tolist(), t))
    dist.destroy_process_group()


def test_gloo_world2_reduction_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in ps:
        pr.start()
    res = [q.get(timeout=240) for _ in ps]
    for pr in ps:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = rempi_amd.default_gen_params(world_size=16, events_per_rank=3000)
    recs = comp = 0
    for r in range(4):
        h = rempi_amd.generate_host(p, r)
        recs += h.shape[0]
        comp += len(O.encode(h, 4096)[0])
    for _, c, t in res:
        assert c == [float(recs), float(comp), 0.0]
        assert t == 2.0  # max over ranks
